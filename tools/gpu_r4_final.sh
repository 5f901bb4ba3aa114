# Round-4 verification on one MI355X, as the driver runs it: the GPU test suite, smoke(), the default
# bench line (N = 1, every extra key).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/fin_tests.log 2>&1
rc=$?; tail -6 gpurun_out/fin_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/fin_bench.log 2>&1 || { tail -20 gpurun_out/fin_bench.log; exit 1; }
grep '^{' gpurun_out/fin_bench.log | tail -1 > gpurun_out/fin_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/fin_bench.json'))
print({k: d[k] for k in ('value','ms_per_step','gpt2_4stage_decode_ms_per_step','gpt2_4stage_prefill_tok_s','llama3_8b_8stage_b32_decode_ms_per_step','gpt2xl_fp8_8stage_b64_decode_ms_per_step','gpt2xl_fp8_8stage_b64_prefill_tok_s') if k in d})"
