#!/bin/bash
# Kernel-boundary cost (tools/rocprof_gaps.py) of the GPT-2 4-stage B=64 and
# Llama-3 8B fp8 B=1 decode graphs: gpurun_out/dec_{gpt2,llama}_gaps.md
set -o pipefail
export TMPDIR=/tmp
G="bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1"
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gp_gpt2 -o run -- python3 $G > gpurun_out/gp_gpt2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gp_llama -o run -- python3 $L > gpurun_out/gp_llama.log 2>&1
rc=$?
for k in gpt2 llama; do
  [ -d gpurun_out/gp_$k ] && python3 tools/rocprof_gaps.py gpurun_out/gp_$k > gpurun_out/dec_${k}_gaps.md
done
rm -rf gpurun_out/gp_gpt2 gpurun_out/gp_llama
exit $rc
