# Current per-kernel table for Llama-3 8B B=32 decode (bf16).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p30 -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/p30.log 2>&1; echo rc=$?
