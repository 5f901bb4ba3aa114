# Round 5: one-shot prefetch race fix (sched_barrier before the image DMA, branch-free operand loads):
# determinism probe, decode GEMM tests, epilogue-prefetch A/B again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python bench/probes/epi_pre_diff.py > gpurun_out/r5r_diff.jsonl 2> gpurun_out/r5r.err || { echo DIFF_FAILED; tail -20 gpurun_out/r5r.err; exit 1; }
cat gpurun_out/r5r_diff.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stream_gemm_gpu.py tests/test_transformer_gpu.py tests/test_head_gpu.py > gpurun_out/r5r_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5r_tests.log; exit 1; }
tail -2 gpurun_out/r5r_tests.log
timeout -k 10 300 python bench/probes/decode_ab.py --switch epi_pre --values 0,1 --rounds 3 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5r_ab_gpt2.jsonl 2> gpurun_out/r5r_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5r_ab.err; exit 1; }
cat gpurun_out/r5r_ab_gpt2.jsonl
timeout -k 10 400 python bench/probes/decode_ab.py --switch epi_pre --values 0,1 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5r_ab_xl.jsonl 2>> gpurun_out/r5r_ab.err || { echo AB2_FAILED; tail -20 gpurun_out/r5r_ab.err; exit 1; }
cat gpurun_out/r5r_ab_xl.jsonl
