#!/bin/bash
# Row-split argmax: numerics, then in-process decode A/B (GPT-2 4-stage B=64,
# Llama-3 8B fp8 B=1, GPT-2 XL fp8 B=64).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/argmax_tests.log 2>&1
rc=$?; tail -3 gpurun_out/argmax_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/argmax_ab.jsonl; : > $out
ab() { timeout -k 10 300 python -u bench/decode_ab.py --switch argmax_split --values 0,1 "$@" >> $out 2> gpurun_out/argmax_ab.err; }
ab --steps 32 --warmup 4 --prefill_iters 1 &&
ab --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 32 --warmup 4 --prefill_iters 1 &&
ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1
rc=$?; cat $out; exit $rc
