# skinny GEMM numerics + decode benches
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -x -q > gpurun_out/tests5.log 2>&1; rc=$?; tail -5 gpurun_out/tests5.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 > gpurun_out/gpt_b1.log 2>&1 && tail -1 gpurun_out/gpt_b1.log &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/gpt_b64.log 2>&1 && tail -1 gpurun_out/gpt_b64.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 > gpurun_out/llama_b32.log 2>&1 && tail -1 gpurun_out/llama_b32.log &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/llama_b1.log 2>&1 && tail -1 gpurun_out/llama_b1.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/xl_fp8_b64.log 2>&1 && tail -1 gpurun_out/xl_fp8_b64.log
