set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/t4.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t4.log
tail -4 gpurun_out/t4.log
timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/gpt1.log 2>&1; tail -3 gpurun_out/gpt1.log
timeout -k 10 300 python bench/gpt_bench.py --batch 16 --prompt 128 --steps 32 >> gpurun_out/gpt1.log 2>&1; tail -1 gpurun_out/gpt1.log
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --dtype fp8 >> gpurun_out/gpt1.log 2>&1; tail -1 gpurun_out/gpt1.log
