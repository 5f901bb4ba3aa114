set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_tests.log 2>&1
rc=$?; tail -2 gpurun_out/v_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || { tail -5 gpurun_out/v_smoke.log; exit 1; }
tail -1 gpurun_out/v_smoke.log | cut -c1-160
timeout -k 10 500 python bench.py > gpurun_out/v_bench.log 2>&1 || { tail -5 gpurun_out/v_bench.log; exit 1; }
tail -1 gpurun_out/v_bench.log
