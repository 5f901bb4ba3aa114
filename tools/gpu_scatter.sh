#!/bin/bash
# QKV scatter prefill: tests, then in-process A/B of GPT-2 prefill (4-stage B=64).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kv8_gpu.py tests/test_pipeline_gpu.py tests/test_fold_norm.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/scatter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/scatter_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/decode_ab.py --switch qkv_scatter --values 0,1 --rounds 3 --steps 4 --warmup 1 --prefill_iters 5 \
  > gpurun_out/scatter_ab.jsonl 2> gpurun_out/scatter_ab.err
rc=$?; cat gpurun_out/scatter_ab.jsonl; exit $rc
