# Re-fit sweep with fragment-order weights (pipes 4-7: shuffled, +pipeline, +M split).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 500 python bench/skinny_sweep.py --m 1,32 --w8 0,1 --shapes llama --iters 10 --pipes 4,5,6,7 --shuf > gpurun_out/sw13_llama.jsonl 2>&1 &&
timeout -k 10 500 python bench/skinny_sweep.py --m 64 --w8 0 --shapes gpt2 --iters 20 --pipes 4,5,6,7 --shuf > gpurun_out/sw13_gpt2.jsonl 2>&1 &&
timeout -k 10 500 python bench/skinny_sweep.py --m 64 --w8 1 --shapes gpt2xl --iters 10 --pipes 4,5,6,7 --shuf > gpurun_out/sw13_xl.jsonl 2>&1
