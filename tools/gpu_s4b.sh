mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof -o run -- python3 bench.py --steps 10 --latency_iters 10 > gpurun_out/cprof.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof32 -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/lprof32.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof64 -o run -- python3 bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/gprof64.log 2>&1; echo rc=$?
