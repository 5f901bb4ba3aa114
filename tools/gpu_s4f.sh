mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xlprof2 -o run -- python3 bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --steps 8 --warmup 2 --prefill_iters 1 --no_graph --dtype fp8 > gpurun_out/xlprof2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof32g -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/lprof32g.log 2>&1; echo rc=$?
