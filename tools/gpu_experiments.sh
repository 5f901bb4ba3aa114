#!/bin/bash
# One-off GPU measurements behind the numbers recorded in profiles/ (run through
# gpurun from the repo root):  bash tools/gpu_experiments.sh <case>
# Every GPU step has its own time limit and the steps of a case are chained, so
# the first failure ends it.  Cases:
#   argmax_ab        row-split argmax: numerics, then in-process decode A/B
#   decode_ab        in-process A/B: bf16 skinny row limit 32 (tile path for wide-N heads at M 33-64) vs 64
#   decode_check     decode projection tests, Llama-3 8B B=1 fp8 / bf16 decode benches
#   flash_check      flash / decode attention tests, flash-vs-SDPA bench, GPT-2 prefill
#   gemm_epi         GEMM epilogue cost on the GPT-2 prefill shapes: bias / +GELU / +residual (separate, in place)
#   kv8              fp8 (e4m3) KV cache: numerics, then GPT-2 / GPT-2 XL decode, bf16 vs fp8 cache
#   kv8_ab           fp8-KV decode attention rows in flight per thread: 10 vs 8 (in-process A/B).
#   kv8g             fp8 KV for GQA / RoPE (Llama-3): tests, then Llama-3 8B B=32 decode bf16 vs fp8 KV.
#   prof_argmax      Llama-3 8B fp8 B=1 decode kernel gaps with the split argmax
#   prof_llama_b32   Llama-3 8B bf16 B=32 decode kernel table + gaps, M=32 projection sweep
#   scatter3         QKV scatter prefill: tests, in-process A/B, per-layer prefill sequence
#   prof_kv8         GPT-2 B=64 decode with the e4m3 KV cache: kernel table + gaps
#   tail_check       kernel + transformer + pipeline GPU tests, smoke, decode benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

case_argmax_ab() {
  # Row-split argmax: numerics, then in-process decode A/B (GPT-2 4-stage B=64,
  # Llama-3 8B fp8 B=1, GPT-2 XL fp8 B=64).
  timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/argmax_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/argmax_tests.log; [ $rc -eq 0 ] || return $rc
  out=gpurun_out/argmax_ab.jsonl; : > $out
  ab() { timeout -k 10 300 python -u bench/probes/decode_ab.py --switch argmax_split --values 0,1 "$@" >> $out 2> gpurun_out/argmax_ab.err; }
  ab --steps 32 --warmup 4 --prefill_iters 1 &&
  ab --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 32 --warmup 4 --prefill_iters 1 &&
  ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1
  rc=$?; cat $out; return $rc
}

case_decode_ab() {
  # in-process A/B: bf16 skinny row limit 32 (tile path for wide-N heads at M 33-64) vs 64
  out=gpurun_out/decode_ab.jsonl
  : > $out
  timeout -k 10 300 python bench/probes/decode_ab.py --switch skinny_max_m --values 32,64 --steps 32 --warmup 4 --prefill_iters 1 >> $out 2>gpurun_out/dab.err &&
  timeout -k 10 400 python bench/probes/decode_ab.py --switch skinny_max_m --values 32,64 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 >> $out 2>>gpurun_out/dab.err
  rc=$?; cat $out; return $rc
}

case_decode_check() {
  timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "shuffled or skinny or w8 or norm or stage" > gpurun_out/pytest_tf.log 2>&1; tail -2 gpurun_out/pytest_tf.log
  timeout -k 10 300 python -u bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 > gpurun_out/llama_fp8_b1.log 2>&1; tail -1 gpurun_out/llama_fp8_b1.log
  timeout -k 10 300 python -u bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 > gpurun_out/llama_bf16_b1.log 2>&1; tail -1 gpurun_out/llama_bf16_b1.log
}

case_flash_check() {
  # flash / decode attention tests, flash-vs-SDPA bench, GPT-2 prefill
  timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or stage or gpt2_small or forward" > gpurun_out/fl_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/fl_tests.log; [ $rc -eq 0 ] || return $rc
  timeout -k 10 200 python bench/probes/flash_bench.py > gpurun_out/flash.jsonl 2>&1; rc=$?; grep '^{' gpurun_out/flash.jsonl | cut -c1-200; [ $rc -eq 0 ] || return $rc
  timeout -k 10 200 python bench/gpt_bench.py --steps 8 --warmup 2 --prefill_iters 5 > gpurun_out/gb.log 2>&1 && tail -1 gpurun_out/gb.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('prefill', d['prefill_tokens_per_s'], 'decode ms', d['ms_per_step'])"
}

case_gemm_epi() {
  # GEMM epilogue cost on the GPT-2 prefill shapes: bias / +GELU / +residual (separate, in place)
  N768=32768x768x768,32768x768x3072
  timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768,$N768 --act none --torch > gpurun_out/ge.jsonl 2>&1 &&
  timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768 --act gelu >> gpurun_out/ge.jsonl 2>&1 &&
  timeout -k 10 120 python bench/gemm_bench.py --shapes $N768 --residual >> gpurun_out/ge.jsonl 2>&1 &&
  timeout -k 10 120 python bench/gemm_bench.py --shapes $N768 --inplace >> gpurun_out/ge.jsonl 2>&1 &&
  timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768,$N768 --act none >> gpurun_out/ge.jsonl 2>&1
  rc=$?; grep '^{' gpurun_out/ge.jsonl; return $rc
}

case_kv8() {
  # fp8 (e4m3) KV cache: numerics, attention regression, then GPT-2 decode with
  # bf16 vs fp8 caches (B=64, B=256) and GPT-2 XL fp8 weights + fp8 cache.
  timeout -k 10 300 python -u -m pytest tests/test_kv8_gpu.py tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/kv8_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/kv8_tests.log; [ $rc -eq 0 ] || return $rc
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
  "; return $rc
}

case_kv8_ab() {
  # fp8-KV decode attention rows in flight per thread: 10 vs 8 (in-process A/B).
  timeout -k 10 200 python -u -m pytest tests/test_kv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/kv8u_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/kv8u_tests.log; [ $rc -eq 0 ] || return $rc
  out=gpurun_out/kv8u_ab.jsonl; : > $out
  ab() { timeout -k 10 300 python -u bench/probes/decode_ab.py --switch kv8_u --values 8,10 "$@" >> $out 2> gpurun_out/kv8u_ab.err; }
  ab --steps 32 --warmup 4 --prefill_iters 1 --kv fp8 &&
  ab --batch 256 --steps 32 --warmup 4 --prefill_iters 1 --kv fp8 &&
  ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --kv fp8 --steps 16 --warmup 2 --prefill_iters 1
  rc=$?; cat $out; return $rc
}

case_kv8g() {
  # fp8 KV for GQA / RoPE (Llama-3): tests, then Llama-3 8B B=32 decode bf16 vs fp8 KV.
  timeout -k 10 300 python -u -m pytest tests/test_kv8_gpu.py tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/kv8g_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/kv8g_tests.log; [ $rc -eq 0 ] || return $rc
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
  "; return $rc
}

case_prof_argmax() {
  L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_amx -o run -- python3 $L > gpurun_out/prof_amx.log 2>&1 &&
  python3 tools/rocprof_gaps.py gpurun_out/prof_amx > gpurun_out/amx_gaps.md
  rc=$?; rm -rf gpurun_out/prof_amx; head -14 gpurun_out/amx_gaps.md; return $rc
}

case_prof_llama_b32() {
  # Llama-3 8B bf16 8-stage B=32 decode (BASELINE config 4, colocated): kernel
  # table + decode-region gaps, and the M=32 projection sweep (bf16 weights).
  L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l32 -o run -- python3 $L > gpurun_out/prof_l32.log 2>&1 &&
  python3 tools/rocprof_summary.py gpurun_out/prof_l32 > gpurun_out/l32_kernels.md &&
  python3 tools/rocprof_gaps.py gpurun_out/prof_l32 > gpurun_out/l32_gaps.md
  rc=$?
  rm -rf gpurun_out/prof_l32
  [ $rc -eq 0 ] || return $rc
  timeout -k 10 400 python3 -u bench/skinny_sweep.py --m 32 --w8 0 --shapes llama --iters 10 > gpurun_out/l32_sweep.jsonl 2> gpurun_out/l32_sweep.err
}

case_scatter3() {
  timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q -k "scatter or gpt2 or golden" \
    --timeout 120 --timeout-method thread > gpurun_out/scatter3_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/scatter3_tests.log; [ $rc -eq 0 ] || return $rc
  timeout -k 10 400 python -u bench/probes/decode_ab.py --switch qkv_scatter --values 0,1 --rounds 3 --steps 4 --warmup 1 --prefill_iters 5 \
    > gpurun_out/scatter3_ab.jsonl 2> gpurun_out/scatter3_ab.err && cat gpurun_out/scatter3_ab.jsonl &&
  bash tools/gpu_prof_prefill.sh && head -8 gpurun_out/prefill_seq.md
}

case_tail_check() {
  # kernel + transformer + pipeline GPU tests, smoke, decode benches
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || return $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; return 1; }
  tail -1 gpurun_out/smoke.log | cut -c1-150
  bash tools/gpu_decode_bench.sh
}

case_prof_kv8() {
  # GPT-2 4-stage B=64 decode with the e4m3 KV cache: kernel table + gaps
  G="bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1 --kv fp8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kv8 -o run -- python3 $G > gpurun_out/prof_kv8.log 2>&1 &&
  python3 tools/rocprof_summary.py gpurun_out/prof_kv8 > gpurun_out/kv8_kernels.md &&
  python3 tools/rocprof_gaps.py gpurun_out/prof_kv8 > gpurun_out/kv8_gaps.md
  rc=$?; rm -rf gpurun_out/prof_kv8; head -8 gpurun_out/kv8_gaps.md; return $rc
}

c=${1:-}
if ! declare -F "case_$c" > /dev/null; then
  echo "usage: $0 <case>; cases: argmax_ab decode_ab decode_check flash_check gemm_epi kv8 kv8_ab kv8g prof_argmax prof_llama_b32 scatter3 prof_kv8 tail_check"; exit 2
fi
"case_$c"
