# 128^2 GEMM unrolled by two: GEMM tests + GEMM bench (tile128 column).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/t20_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t20_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gemm_bench.py --shapes 65536x512x4096,16384x512x4096,32768x768x768,32768x768x3072,4096x4096x4096,8192x8192x8192,2048x2304x768 > gpurun_out/t20_gemm.jsonl 2>&1 && cat gpurun_out/t20_gemm.jsonl
