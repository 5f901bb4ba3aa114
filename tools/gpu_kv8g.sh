#!/bin/bash
# fp8 KV for GQA / RoPE (Llama-3): tests, then Llama-3 8B B=32 decode bf16 vs fp8 KV.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kv8_gpu.py tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/kv8g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/kv8g_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/kv8g_bench.jsonl; : > $out
run() { timeout -k 10 300 python -u bench/gpt_bench.py "$@" > gpurun_out/kv8g_b.log 2>&1 && tail -1 gpurun_out/kv8g_b.log >> $out; }
run --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 --kv fp8 &&
run --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 &&
run --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --kv fp8 --steps 32 --warmup 4 --prefill_iters 1
rc=$?; python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); c=d['config']
    print(c['model'], 'B=%d'%c['micro_batch'], d['dtype'][-22:], 'ms/step %.4f'%d['ms_per_step'], 'tok/s %.0f'%d['value'], 'prefill %.0f'%d['prefill_tokens_per_s'])
"; exit $rc
