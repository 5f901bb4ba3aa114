export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q -k "gemm or fp8 or stage" > gpurun_out/tests6.log 2>&1; rc=$?; tail -2 gpurun_out/tests6.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python bench/skinny_sweep.py --m 1,32,64 > gpurun_out/skinny_sweep2.jsonl 2>&1 && cut -c1-300 gpurun_out/skinny_sweep2.jsonl &&
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 > gpurun_out/gpt_b1.log 2>&1 && tail -1 gpurun_out/gpt_b1.log | cut -c1-200 &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 > gpurun_out/llama_b32.log 2>&1 && tail -1 gpurun_out/llama_b32.log | cut -c1-200 &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/llama_b1.log 2>&1 && tail -1 gpurun_out/llama_b1.log | cut -c1-200 &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/xl_fp8_b64.log 2>&1 && tail -1 gpurun_out/xl_fp8_b64.log | cut -c1-200
