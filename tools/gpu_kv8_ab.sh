#!/bin/bash
# fp8-KV decode attention rows in flight per thread: 10 vs 8 (in-process A/B).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/kv8u_tests.log 2>&1
rc=$?; tail -2 gpurun_out/kv8u_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/kv8u_ab.jsonl; : > $out
ab() { timeout -k 10 300 python -u bench/decode_ab.py --switch kv8_u --values 8,10 "$@" >> $out 2> gpurun_out/kv8u_ab.err; }
ab --steps 32 --warmup 4 --prefill_iters 1 --kv fp8 &&
ab --batch 256 --steps 32 --warmup 4 --prefill_iters 1 --kv fp8 &&
ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --kv fp8 --steps 16 --warmup 2 --prefill_iters 1
rc=$?; cat $out; exit $rc
