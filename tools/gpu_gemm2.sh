# GEMM numerics + A/B, transformer tests, B=1 decode, flagship bench.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q > gpurun_out/tests2.log 2>&1; rc=$?; tail -3 gpurun_out/tests2.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench2.jsonl 2>&1 && cat gpurun_out/gemm_bench2.jsonl &&
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 > gpurun_out/gpt_b1.log 2>&1 && tail -1 gpurun_out/gpt_b1.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1 && tail -1 gpurun_out/bench_n1.log
