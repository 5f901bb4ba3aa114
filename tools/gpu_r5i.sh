# Round 5: full GPU suite, decode GEMM epilogue-prefetch A/B, norm_q8 probe (R=1), XL prefill, GPT-2 decode gaps detail.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5i_tests.log; exit 1; }
tail -3 gpurun_out/r5i_tests.log
timeout -k 10 300 python bench/probes/decode_ab.py --switch epi_pre --values 0,1 --rounds 3 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5i_ab_epi_gpt2.jsonl 2> gpurun_out/r5i_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5i_ab.err; exit 1; }
cat gpurun_out/r5i_ab_epi_gpt2.jsonl
timeout -k 10 400 python bench/probes/decode_ab.py --switch epi_pre --values 0,1 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5i_ab_epi_xl.jsonl 2>> gpurun_out/r5i_ab.err || { echo AB2_FAILED; tail -20 gpurun_out/r5i_ab.err; exit 1; }
cat gpurun_out/r5i_ab_epi_xl.jsonl
timeout -k 10 200 python bench/probes/norm_q8_probe.py > gpurun_out/r5i_normq8.jsonl 2> gpurun_out/r5i_normq8.err || { echo PROBE_FAILED; tail -20 gpurun_out/r5i_normq8.err; exit 1; }
cat gpurun_out/r5i_normq8.jsonl
G="bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gp_gpt2 -o run -- python3 $G > gpurun_out/gp_gpt2.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/gp_gpt2.log; exit 1; }
python3 tools/rocprof_gaps.py gpurun_out/gp_gpt2 > gpurun_out/r5i_gpt2_b64_decode_gaps.md
rm -rf gpurun_out/gp_gpt2
head -18 gpurun_out/r5i_gpt2_b64_decode_gaps.md
