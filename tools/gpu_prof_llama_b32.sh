#!/bin/bash
# Llama-3 8B bf16 8-stage B=32 decode (BASELINE config 4, colocated): kernel
# table + decode-region gaps, and the M=32 projection sweep (bf16 weights).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l32 -o run -- python3 $L > gpurun_out/prof_l32.log 2>&1 &&
python3 tools/rocprof_summary.py gpurun_out/prof_l32 > gpurun_out/l32_kernels.md &&
python3 tools/rocprof_gaps.py gpurun_out/prof_l32 > gpurun_out/l32_gaps.md
rc=$?
rm -rf gpurun_out/prof_l32
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench/skinny_sweep.py --m 32 --w8 0 --shapes llama --iters 10 > gpurun_out/l32_sweep.jsonl 2> gpurun_out/l32_sweep.err
