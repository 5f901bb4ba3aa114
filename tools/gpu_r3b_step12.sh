# round 3 session 2, step 12: GPT-2 prefill GEMM shapes, 128^2 vs 256^2 tiles vs hipBLASLt, with the pipeline's epilogues
set -o pipefail
export TMPDIR=/tmp
S=32768x3072x768,32768x768x3072,32768x2304x768,32768x768x768
timeout -k 10 200 python -u bench/gemm_bench.py --shapes $S --torch > gpurun_out/s12_none.jsonl 2>/dev/null &&
timeout -k 10 200 python -u bench/gemm_bench.py --shapes 32768x3072x768 --act gelu --torch > gpurun_out/s12_gelu.jsonl 2>/dev/null &&
timeout -k 10 200 python -u bench/gemm_bench.py --shapes 32768x768x3072,32768x768x768 --inplace > gpurun_out/s12_res.jsonl 2>/dev/null
rc=$?; cat gpurun_out/s12_*.jsonl; exit $rc
