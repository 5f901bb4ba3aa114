# round 3 (second session): GPU tests, smoke, driver bench line on the rebuilt library
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r3b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3b_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r3b_smoke.log | cut -c1-160
timeout -k 10 600 python -u bench.py > gpurun_out/r3b_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3b_bench.log | cut -c1-400
