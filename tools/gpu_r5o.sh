# Round 5 final check: full GPU suite, smoke(), the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5o_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5o_tests.log; exit 1; }
tail -3 gpurun_out/r5o_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5o_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r5o_smoke.log; exit 1; }
tail -1 gpurun_out/r5o_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5o_bench.json 2> gpurun_out/r5o_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5o_bench.err; exit 1; }
cat gpurun_out/r5o_bench.json
