export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s4e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s4e_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 > gpurun_out/s4e_llama_b1_fp8.log 2>&1 && tail -1 gpurun_out/s4e_llama_b1_fp8.log &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype fp8 > gpurun_out/s4e_llama_b32_fp8.log 2>&1 && tail -1 gpurun_out/s4e_llama_b32_fp8.log &&
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 > gpurun_out/s4e_gpt2xl_fp8.log 2>&1 && tail -1 gpurun_out/s4e_gpt2xl_fp8.log
