# Round-4 GPU step 8: one-round-trip decode combine; the one-pass decode attention with 2 / 3 key
# splits on Llama-3 8B B=32 (two workgroups per CU now fit the 76 KiB of LDS) — attention tests, decode A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kv8_gpu.py tests/test_transformer_gpu.py -k "attn or kv8 or decode" -q --timeout 120 \
  --timeout-method thread -x > gpurun_out/s8_tests.log 2>&1 || { tail -40 gpurun_out/s8_tests.log; exit 1; }
tail -2 gpurun_out/s8_tests.log
L="--model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch decode_1p_ns --values 0,2,3 --rounds 2 $L \
  > gpurun_out/s8_ab_ns_llama.jsonl 2> gpurun_out/s8_ab.err || exit 1
tail -1 gpurun_out/s8_ab_ns_llama.jsonl | cut -c1-400
