#!/bin/bash
# GEMM epilogue cost on the GPT-2 prefill shapes: bias / +GELU / +residual (separate, in place)
set -o pipefail
N768=32768x768x768,32768x768x3072
timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768,$N768 --act none --torch > gpurun_out/ge.jsonl 2>&1 &&
timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768 --act gelu >> gpurun_out/ge.jsonl 2>&1 &&
timeout -k 10 120 python bench/gemm_bench.py --shapes $N768 --residual >> gpurun_out/ge.jsonl 2>&1 &&
timeout -k 10 120 python bench/gemm_bench.py --shapes $N768 --inplace >> gpurun_out/ge.jsonl 2>&1 &&
timeout -k 10 120 python bench/gemm_bench.py --shapes 32768x3072x768,$N768 --act none >> gpurun_out/ge.jsonl 2>&1
rc=$?; grep '^{' gpurun_out/ge.jsonl; exit $rc
