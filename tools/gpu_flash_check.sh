#!/bin/bash
# flash / decode attention tests, flash-vs-SDPA bench, GPT-2 prefill
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or stage or gpt2_small or forward" > gpurun_out/fl_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fl_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/flash_bench.py > gpurun_out/flash.jsonl 2>&1; rc=$?; grep '^{' gpurun_out/flash.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/gpt_bench.py --steps 8 --warmup 2 --prefill_iters 5 > gpurun_out/gb.log 2>&1 && tail -1 gpurun_out/gb.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('prefill', d['prefill_tokens_per_s'], 'decode ms', d['ms_per_step'])"
