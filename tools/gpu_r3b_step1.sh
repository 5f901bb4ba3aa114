# round 3 session 2, step 1: one-pass decode attention — correctness, in-process A/B, then full verification
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/s1_dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s1_dec_tests.log; [ $rc -eq 0 ] || exit $rc
ab() { timeout -k 10 400 python -u bench/probes/decode_ab.py --switch decode_1p --values 0,1 "$@" >> gpurun_out/s1_ab.jsonl 2> gpurun_out/s1_ab.err && tail -1 gpurun_out/s1_ab.jsonl; }
: > gpurun_out/s1_ab.jsonl
ab --model gpt2 --stages 4 --batch 64 --prompt 512 &&
ab --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 &&
ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/s1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s1_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/s1_smoke.log | cut -c1-160
