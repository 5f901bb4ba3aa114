# 256^2 GEMM K-loop unrolled by two (static LDS offsets): GEMM tests + GEMM bench + flagship + GPT-2 prefill.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/u17_tests.log 2>&1; rc=$?; tail -2 gpurun_out/u17_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gemm_bench.py --shapes 65536x512x4096,32768x2304x768,32768x3072x768,32768x768x3072,4096x4096x4096,8192x8192x8192,16384x6144x4096,16384x28672x4096,16384x4096x14336 > gpurun_out/u17_gemm.jsonl 2>&1 && cat gpurun_out/u17_gemm.jsonl &&
timeout -k 10 300 python bench.py > gpurun_out/u17_bench.log 2>&1 && tail -1 gpurun_out/u17_bench.log &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 8 > gpurun_out/u17_gpt2.log 2>&1 && tail -1 gpurun_out/u17_gpt2.log
