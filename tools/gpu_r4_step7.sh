# Round-4 GPU step 7: one-shot GEMM with the row statistics taken while the weights are in flight —
# its tests, the folded-norm A/B (in-kernel statistics cost), the GPT-2 / XL decode transformer tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream_gemm_gpu.py tests/test_head_gpu.py -q --timeout 120 \
  --timeout-method thread -x > gpurun_out/s7_tests.log 2>&1 || { tail -40 gpurun_out/s7_tests.log; exit 1; }
tail -2 gpurun_out/s7_tests.log
timeout -k 10 300 python -u bench/oneshot_sweep.py --shapes gpt2,gpt2xl --epi ln,ln_gelu > gpurun_out/s7_epi.jsonl 2> gpurun_out/s7_epi.err || exit 1
grep "^{" gpurun_out/s7_epi.jsonl | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['N'],d['K'],d['w8'],'plain',d['plain_os1_us'],'ln',d['ln_os1_us'],'ln_gelu',d['ln_gelu_os1_us'],'skinny ln',d['ln_os0_us'])"
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py -q --timeout 300 --timeout-method thread -x \
  -k "gpt2 or xl" > gpurun_out/s7_tf_tests.log 2>&1 || { tail -40 gpurun_out/s7_tf_tests.log; exit 1; }
tail -2 gpurun_out/s7_tf_tests.log
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 2 $G \
  > gpurun_out/s7_ab_os_gpt2.jsonl 2> gpurun_out/s7_ab.err || exit 1
tail -1 gpurun_out/s7_ab_os_gpt2.jsonl | cut -c1-300
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 2 $X \
  > gpurun_out/s7_ab_os_xl.jsonl 2>> gpurun_out/s7_ab.err || exit 1
tail -1 gpurun_out/s7_ab_os_xl.jsonl | cut -c1-300
