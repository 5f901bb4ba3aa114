# Round-4 GPU step 10: where the prefill tail split lands in the GPT-2 pipeline (kernel table, split on / off).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_on -o run -- python3 $G > gpurun_out/prof_on.log 2>&1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/prof_on > gpurun_out/s10_prefill_split_on.md
rm -rf gpurun_out/prof_on
DNN_SPLIT_TAIL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_off -o run -- python3 $G > gpurun_out/prof_off.log 2>&1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/prof_off > gpurun_out/s10_prefill_split_off.md
rm -rf gpurun_out/prof_off
grep "gemm_bf16_256" gpurun_out/s10_prefill_split_on.md | cut -c1-160
echo ---
grep "gemm_bf16_256" gpurun_out/s10_prefill_split_off.md | cut -c1-160
