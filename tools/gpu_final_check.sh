#!/bin/bash
# Round verification: all GPU tests, smoke, the driver's default bench line,
# a rocprof kernel table of the headline bench, and the decode benches.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log | cut -c1-120
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 10 --warmup 3 --no_extra > gpurun_out/prof_final.log 2>&1 &&
python3 tools/rocprof_summary.py gpurun_out/prof_final > gpurun_out/final_kernels.md && rm -rf gpurun_out/prof_final
bash tools/gpu_decode_bench.sh
