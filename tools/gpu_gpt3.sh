export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_transformer_gpu.py -q -x > gpurun_out/t7.log 2>&1; tail -1 gpurun_out/t7.log
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 2>&1 | grep metric
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 2>&1 | grep metric
timeout -k 10 300 python bench/gpt_bench.py --batch 256 --prompt 256 2>&1 | grep metric
