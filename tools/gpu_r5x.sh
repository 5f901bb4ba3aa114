# Round 5 final check after the one-shot image-sync fix: full GPU suite, smoke(), the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5x_tests.log; exit 1; }
tail -3 gpurun_out/r5x_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5x_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r5x_smoke.log; exit 1; }
tail -1 gpurun_out/r5x_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5x_bench.json 2> gpurun_out/r5x_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5x_bench.err; exit 1; }
cat gpurun_out/r5x_bench.json
