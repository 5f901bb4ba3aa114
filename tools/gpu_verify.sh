# Round-end style verification on one MI355X: GPU tests, smoke, flagship bench, kernel profile.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/tests_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench.log 2>&1 && tail -1 gpurun_out/prof_bench.log
