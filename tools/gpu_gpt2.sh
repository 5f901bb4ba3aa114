mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 > gpurun_out/gpt2.log 2>&1; grep -v amdgpu.ids gpurun_out/gpt2.log | tail -2
timeout -k 10 300 python bench/gpt_bench.py --batch 256 --prompt 256 --steps 32 >> gpurun_out/gpt2.log 2>&1; tail -1 gpurun_out/gpt2.log
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 >> gpurun_out/gpt2.log 2>&1; tail -1 gpurun_out/gpt2.log
