# Round 5: PMC passes over the GPT-2 4-stage B=64 decode on the final library (one-shot image sync + LDS floor).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_pmc.sh gpurun_out/pmc_g5 bench/gpt_bench.py --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_g5/p1.log; tail -20 gpurun_out/pmc_g5/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_g5 --top 14 > gpurun_out/r5cc_pmc_gpt2_decode.md
rm -rf gpurun_out/pmc_g5/p1 gpurun_out/pmc_g5/p2
tail -18 gpurun_out/r5cc_pmc_gpt2_decode.md
