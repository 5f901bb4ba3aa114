export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s4h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s4h_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 > gpurun_out/s4h_xl.log 2>&1 && tail -1 gpurun_out/s4h_xl.log &&
timeout -k 10 300 python bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 > gpurun_out/s4h_gpt2.log 2>&1 && tail -1 gpurun_out/s4h_gpt2.log &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 > gpurun_out/s4h_l32.log 2>&1 && tail -1 gpurun_out/s4h_l32.log &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 > gpurun_out/s4h_l1.log 2>&1 && tail -1 gpurun_out/s4h_l1.log
