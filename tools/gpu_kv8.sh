#!/bin/bash
# fp8 (e4m3) KV cache: numerics, attention regression, then GPT-2 decode with
# bf16 vs fp8 caches (B=64, B=256) and GPT-2 XL fp8 weights + fp8 cache.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kv8_gpu.py tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/kv8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/kv8_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/kv8_bench.jsonl; : > $out
run() { timeout -k 10 300 python -u bench/gpt_bench.py "$@" > gpurun_out/kv8_b.log 2>&1 && tail -1 gpurun_out/kv8_b.log >> $out; }
run --batch 64 --prompt 512 --prefill_iters 1 --kv fp8 &&
run --batch 64 --prompt 512 --prefill_iters 1 &&
run --batch 256 --prompt 512 --prefill_iters 1 --kv fp8 &&
run --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --kv fp8 --steps 16 --warmup 2 --prefill_iters 1
rc=$?; python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); c=d['config']
    print(c['model'], 'B=%d'%c['micro_batch'], d['dtype'][-20:], 'ms/step %.4f'%d['ms_per_step'], 'tok/s %.0f'%d['value'], 'prefill %.0f'%d['prefill_tokens_per_s'])
"; exit $rc
