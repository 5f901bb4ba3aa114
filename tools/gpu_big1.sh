# Llama-3 8B 8-stage bf16 and GPT-2 XL 8-stage fp8, colocated on 1 GPU.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 > gpurun_out/llama_b32.log 2>&1; rc=$?; tail -2 gpurun_out/llama_b32.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/llama_b1.log 2>&1 && tail -1 gpurun_out/llama_b1.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/xl_fp8_b64.log 2>&1 && tail -1 gpurun_out/xl_fp8_b64.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype bf16 --batch 64 --prompt 512 --steps 32 > gpurun_out/xl_bf16_b64.log 2>&1 && tail -1 gpurun_out/xl_bf16_b64.log
