# Round 5: stream-reduce / skinny epilogue prefetch on Llama-3 8B B=32 decode (A/B), decode GEMM tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_stream_gemm_gpu.py tests/test_kernels_gpu.py tests/test_head_gpu.py > gpurun_out/r5j_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5j_tests.log; exit 1; }
tail -2 gpurun_out/r5j_tests.log
timeout -k 10 500 python bench/probes/decode_ab.py --switch epi_pre --values 0,1 --rounds 2 --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5j_ab_epi_llama.jsonl 2> gpurun_out/r5j_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5j_ab.err; exit 1; }
cat gpurun_out/r5j_ab_epi_llama.jsonl
