# Current per-kernel tables for Llama-3 8B B=1 decode, bf16 and fp8 weights.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p27b -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 16 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/p27b.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p27f -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 16 --warmup 2 --prefill_iters 1 --no_graph --dtype fp8 > gpurun_out/p27f.log 2>&1; echo rc=$?
