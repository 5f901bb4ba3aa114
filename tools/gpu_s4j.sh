export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 python bench.py > gpurun_out/s4j_bench.log 2>&1 && tail -1 gpurun_out/s4j_bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof2 -o run -- python3 bench.py --steps 10 --latency_iters 10 > gpurun_out/cprof2.log 2>&1; echo rc=$?
