# Skinny GEMM sweep with M split, graph-timed (device time per launch).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench/skinny_sweep.py --m 32,64 --w8 0 --shapes gpt2 --iters 20 > gpurun_out/sw4_gpt2.jsonl 2>&1 &&
timeout -k 10 500 python bench/skinny_sweep.py --m 32 --w8 0,1 --shapes llama --iters 10 > gpurun_out/sw4_llama.jsonl 2>&1 &&
timeout -k 10 500 python bench/skinny_sweep.py --m 64 --w8 1 --shapes gpt2xl --iters 10 > gpurun_out/sw4_xl.jsonl 2>&1
