#!/bin/bash
# Kernel tables + PMC passes of the decode benchmarks (GPT-2 4-stage B=64 bf16,
# Llama-3 8B B=1 fp8): gpurun_out/prof_dec_{gpt2,llama}/ and pmc_dec_{gpt2,llama}/.
set -o pipefail
export TMPDIR=/tmp
G="bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1"
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec_gpt2 -o run -- python3 $G > gpurun_out/prof_dec_gpt2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec_llama -o run -- python3 $L > gpurun_out/prof_dec_llama.log 2>&1 &&
bash tools/gpu_pmc.sh gpurun_out/pmc_dec_gpt2 $G &&
bash tools/gpu_pmc.sh gpurun_out/pmc_dec_llama $L
rc=$?
# summaries only (the raw rocprof databases exceed what gpurun copies back)
for k in gpt2 llama; do
  [ -d gpurun_out/prof_dec_$k ] && python3 tools/rocprof_summary.py gpurun_out/prof_dec_$k > gpurun_out/dec_${k}_kernels.md
  [ -d gpurun_out/pmc_dec_$k ] && python3 tools/pmc_summary.py gpurun_out/pmc_dec_$k --min_grid 1 --top 8 > gpurun_out/dec_${k}_pmc.md
done
rm -rf gpurun_out/prof_dec_* gpurun_out/pmc_dec_*
exit $rc
