# 256^2 GEMM: numerics, then throughput A/B, then the B=1 decode bench.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1 && tail -3 gpurun_out/gemm_tests.log &&
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench.jsonl 2>&1 && cat gpurun_out/gemm_bench.jsonl &&
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 > gpurun_out/gpt_b1.log 2>&1; rc=$?; tail -15 gpurun_out/gpt_b1.log; exit $rc
