# round 3 session 2, step 4: flash prefetch depth (tests, kernel A/B, prefill A/B)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kv8_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > gpurun_out/s4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/probes/flash_bench.py > gpurun_out/s4_flash.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/s4_flash.log
ab() { timeout -k 10 400 python -u bench/probes/decode_ab.py --switch flash_pf --values 1,2 "$@" >> gpurun_out/s4_ab.jsonl 2> gpurun_out/s4_ab.err && tail -1 gpurun_out/s4_ab.jsonl; }
: > gpurun_out/s4_ab.jsonl
ab --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 4 --warmup 1 &&
ab --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 4 --warmup 1 --prefill_iters 2
