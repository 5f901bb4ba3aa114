mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof1 -o run -- python3 bench/gpt_bench.py --batch 1 --prompt 128 --steps 64 --prefill_iters 1 --no_graph > gpurun_out/gprof1.log 2>&1; echo rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof2 -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 16 --prefill_iters 2 --no_graph > gpurun_out/gprof2.log 2>&1; echo rc=$?
