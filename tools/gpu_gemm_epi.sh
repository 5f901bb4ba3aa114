#!/bin/bash
# GEMM epilogue cost on the GPT-2 prefill shapes (bias / bias+GELU), ours vs torch
set -o pipefail
S=32768x2304x768,32768x768x768,32768x3072x768,32768x768x3072
timeout -k 10 200 python bench/gemm_bench.py --shapes $S --act none > gpurun_out/gemm_epi_none.jsonl 2>&1 &&
timeout -k 10 200 python bench/gemm_bench.py --shapes $S --act gelu > gpurun_out/gemm_epi_gelu.jsonl 2>&1
rc=$?; cat gpurun_out/gemm_epi_*.jsonl | grep '^{'; exit $rc
