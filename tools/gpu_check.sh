#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root):
#   tools/gpu_check.sh [tests|bench|prof|all] [extra pytest -k expr]
# Every GPU step has its own time limit; steps are chained so the first
# failure ends the call.  Output lands in gpurun_out/ (merged back by gpurun).
set -o pipefail
export TMPDIR=/tmp
mode=${1:-all}
kexpr=${2:-}
mkdir -p gpurun_out
run_tests() {
  if [ -n "$kexpr" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr" \
      > gpurun_out/pytest_gpu.log 2>&1
  else
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
  fi
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; return $rc
}
run_bench() {
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  rc=$?; tail -3 gpurun_out/bench.log; return $rc
}
run_prof() {
  rm -rf gpurun_out/prof_bench
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no_extra > gpurun_out/prof_bench.log 2>&1
}
case "$mode" in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && run_bench && run_prof ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
