#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q -k "scatter or gpt2 or golden" \
  --timeout 120 --timeout-method thread > gpurun_out/scatter3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/scatter3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/decode_ab.py --switch qkv_scatter --values 0,1 --rounds 3 --steps 4 --warmup 1 --prefill_iters 5 \
  > gpurun_out/scatter3_ab.jsonl 2> gpurun_out/scatter3_ab.err && cat gpurun_out/scatter3_ab.jsonl &&
bash tools/gpu_prof_prefill.sh && head -8 gpurun_out/prefill_seq.md
