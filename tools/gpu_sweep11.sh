# Pre-shuffled (fragment-order) decode weights vs row-major: graph-timed sweep, Llama-3 8B shapes.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 500 python bench/skinny_sweep.py --m 1,32 --w8 0 --shapes llama --iters 10 --pipes 0,1,4,5 --shuf > gpurun_out/sw11_llama.jsonl 2>&1 &&
timeout -k 10 500 python bench/skinny_sweep.py --m 1,32 --w8 1 --shapes llama --iters 10 --pipes 0,1,4,5 --shuf > gpurun_out/sw11_llama_w8.jsonl 2>&1
