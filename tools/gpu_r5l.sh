# Round 5: epilogue-prefetch bit-identity tests, smoke(), the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream_gemm_gpu.py -k "prefetch or oneshot" > gpurun_out/r5l_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5l_tests.log; exit 1; }
tail -2 gpurun_out/r5l_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5l_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r5l_smoke.log; exit 1; }
tail -3 gpurun_out/r5l_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5l_bench.json 2> gpurun_out/r5l_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5l_bench.err; exit 1; }
cat gpurun_out/r5l_bench.json
