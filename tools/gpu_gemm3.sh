# GEMM epilogue A/B: kernel tests, GEMM throughput (plain and GELU), GPT-2 prefill.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/g3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g3_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/g3_gemm_none.jsonl 2>&1 && cat gpurun_out/g3_gemm_none.jsonl &&
timeout -k 10 300 python bench/gemm_bench.py --act gelu --shapes 32768x3072x768,32768x3072x1600,8192x8192x8192 > gpurun_out/g3_gemm_gelu.jsonl 2>&1 && cat gpurun_out/g3_gemm_gelu.jsonl &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 16 > gpurun_out/g3_gpt2.log 2>&1 && tail -1 gpurun_out/g3_gpt2.log &&
timeout -k 10 300 python bench.py > gpurun_out/g3_bench.log 2>&1 && tail -1 gpurun_out/g3_bench.log
