#!/bin/bash
# QKV scatter prefill incl. fp8 / partial column tiles: tests, then in-process
# A/B of GPT-2 (bf16) and GPT-2 XL (fp8 weights) prefill.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kv8_gpu.py tests/test_pipeline_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/scatter2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/scatter2_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/scatter2_ab.jsonl; : > $out
ab() { timeout -k 10 400 python -u bench/decode_ab.py --switch qkv_scatter --values 0,1 "$@" >> $out 2> gpurun_out/scatter2_ab.err; }
ab --rounds 3 --steps 4 --warmup 1 --prefill_iters 5 &&
ab --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 2
rc=$?; cat $out; exit $rc
