#!/bin/bash
# Persistent 256^2 GEMM: numerics (GEMM / fold-norm / transformer tests), then
# the interleaved in-process A/B (bench/gemm_persist_ab.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fold_norm.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "gemm or fold or norm" > gpurun_out/persist_tests.log 2>&1
rc=$?; tail -3 gpurun_out/persist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/gemm_persist_ab.py > gpurun_out/persist_ab.jsonl 2> gpurun_out/persist_ab.err
rc=$?; cat gpurun_out/persist_ab.jsonl; exit $rc
