#!/bin/bash
# kernel + transformer + pipeline GPU tests, smoke, decode benches
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-150
bash tools/gpu_decode_bench.sh
