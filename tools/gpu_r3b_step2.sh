# round 3 session 2, step 2: one-pass decode attention variants (tests, kernel probe with rotating caches)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2_dec_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/probes/attn_1p_probe.py > gpurun_out/s2_probe.jsonl 2> gpurun_out/s2_probe.err; rc=$?
cat gpurun_out/s2_probe.jsonl; exit $rc
