# round 3 session 2, step 7: flash hd64 LDS fragments requested up front (tests, kernel time, prefill)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kv8_gpu.py -k "flash or prefill or golden" -x -q --timeout 200 --timeout-method thread > gpurun_out/s7_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s7_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/probes/flash_bench.py > gpurun_out/s7_flash.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/s7_flash.log
timeout -k 10 300 python -u bench/gpt_bench.py --steps 4 --warmup 1 --prefill_iters 3 > gpurun_out/s7_gpt2.log 2>&1 || exit 1
tail -1 gpurun_out/s7_gpt2.log | cut -c1-250
