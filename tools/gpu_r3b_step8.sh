# round 3 session 2, step 8: one-pass decode with cooperative exponentials + batched probability reads
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kv8_gpu.py -k "attn_decode or decode" -x -q --timeout 200 --timeout-method thread > gpurun_out/s8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/probes/attn_1p_probe.py --variants batched,1p,1p_kdef > gpurun_out/s8_probe.jsonl 2> gpurun_out/s8_probe.err || exit 1
cat gpurun_out/s8_probe.jsonl
: > gpurun_out/s8_ab.jsonl
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch decode_1p --values 0,1 --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 >> gpurun_out/s8_ab.jsonl 2> gpurun_out/s8_ab.err && tail -1 gpurun_out/s8_ab.jsonl
