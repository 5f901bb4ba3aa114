# round 3 session 2, step 10: one-pass decode defaults (KF for GQA), row-layout scores for GQA probe
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k "attn_decode" -x -q --timeout 200 --timeout-method thread > gpurun_out/s10_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s10_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/probes/attn_1p_probe.py --shapes llama_b32 --variants batched,1p,1p_kf0,1p_rs1 --rounds 3 > gpurun_out/s10_probe.jsonl 2> gpurun_out/s10_probe.err || exit 1
cat gpurun_out/s10_probe.jsonl
