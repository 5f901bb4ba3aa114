# round 3 session 2, step 9: one-pass decode K/V-before-q variant (tests, kernel probe, Llama decode A/B)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k "attn_decode" -x -q --timeout 200 --timeout-method thread > gpurun_out/s9_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s9_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/probes/attn_1p_probe.py > gpurun_out/s9_probe.jsonl 2> gpurun_out/s9_probe.err || exit 1
cat gpurun_out/s9_probe.jsonl
: > gpurun_out/s9_ab.jsonl
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch decode_1p_kf --values 0,1 --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 >> gpurun_out/s9_ab.jsonl 2> gpurun_out/s9_ab.err && tail -1 gpurun_out/s9_ab.jsonl
