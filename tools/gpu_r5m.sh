# Round 5: PMC passes over the GPT-2 XL fp8 8-stage B=64 prefill (MX GEMMs, norm_q8) + decode (one-shot with prefetch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_pmc.sh gpurun_out/pmc_xl5 bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_xl5/p1.log gpurun_out/pmc_xl5/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_xl5 --top 12 > gpurun_out/r5m_pmc_gpt2xl_fp8.md
rm -rf gpurun_out/pmc_xl5/p1 gpurun_out/pmc_xl5/p2
tail -16 gpurun_out/r5m_pmc_gpt2xl_fp8.md
timeout -k 10 300 python bench/probes/oneshot_anatomy.py > gpurun_out/r5m_oneshot_anatomy.jsonl 2> gpurun_out/r5m_anat.err || { echo ANAT_FAILED; tail -20 gpurun_out/r5m_anat.err; exit 1; }
cat gpurun_out/r5m_oneshot_anatomy.jsonl
