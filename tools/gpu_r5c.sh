set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/r5c_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5c_tests.log; exit 1; }
tail -3 gpurun_out/r5c_tests.log
timeout -k 10 300 python bench/probes/ring_host_probe.py --items 256 > gpurun_out/r5c_ring_host.jsonl 2> gpurun_out/r5c_ring_host.err || { echo PROBE_FAILED; tail -20 gpurun_out/r5c_ring_host.err; exit 1; }
cat gpurun_out/r5c_ring_host.jsonl
