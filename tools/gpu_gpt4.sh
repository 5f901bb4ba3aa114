export PYTHONPATH=$PWD
timeout -k 10 300 python bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 2>&1 | tail -5
