# Round-4 final tree (last): GPU suite, smoke, bench line, decode kernel tables of BASELINE configs 3-5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/fin5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/fin5_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin5_smoke.log 2>&1 || { tail -20 gpurun_out/fin5_smoke.log; exit 1; }
tail -1 gpurun_out/fin5_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/fin5_bench.log 2>&1 || { tail -20 gpurun_out/fin5_bench.log; exit 1; }
grep '^{' gpurun_out/fin5_bench.log | tail -1 > gpurun_out/fin5_bench.json
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
for k in gpt2 xl llama; do
  case $k in gpt2) C=$G;; xl) C=$X;; llama) C=$L;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$k -o run -- python3 $C > gpurun_out/prof_$k.log 2>&1 || exit 1
  python3 tools/rocprof_summary.py gpurun_out/prof_$k > gpurun_out/fin5_${k}_kernels.md
  python3 tools/rocprof_gaps.py gpurun_out/prof_$k > gpurun_out/fin5_${k}_gaps.md 2>/dev/null || true
  rm -rf gpurun_out/prof_$k
done
python3 -c "
import json; d=json.load(open('gpurun_out/fin5_bench.json'))
print({k: d[k] for k in ('value','ms_per_step','gpt2_4stage_decode_ms_per_step','gpt2_4stage_prefill_tok_s','llama3_8b_8stage_b32_decode_ms_per_step','gpt2xl_fp8_8stage_b64_decode_ms_per_step','gpt2xl_fp8_8stage_b64_prefill_tok_s') if k in d})"
