# Round 5: kernel tables of the GPT-2 XL fp8 B=64 and Llama-3 8B B=32 decode steps after the epilogue prefetch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
X="bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 32 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k1 -o run -- python3 $X > gpurun_out/prof_k1.log 2>&1 || { echo PROF1_FAILED; tail -20 gpurun_out/prof_k1.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof_k1 > gpurun_out/r5k_gpt2xl_fp8_b64_decode_kernels.md
rm -rf gpurun_out/prof_k1
head -16 gpurun_out/r5k_gpt2xl_fp8_b64_decode_kernels.md
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 --warmup 2 --prefill_iters 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k2 -o run -- python3 $L > gpurun_out/prof_k2.log 2>&1 || { echo PROF2_FAILED; tail -20 gpurun_out/prof_k2.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof_k2 > gpurun_out/r5k_llama8b_b32_decode_kernels.md
rm -rf gpurun_out/prof_k2
head -16 gpurun_out/r5k_llama8b_b32_decode_kernels.md
# two 32-sequence microbatches on two HIP streams vs one of 64 (projection latency under the other lane's attention)
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 32 --microbatches 2 --lanes 2 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5k_xl_lanes.json 2> gpurun_out/r5k_lanes.err || { echo LANES_FAILED; tail -20 gpurun_out/r5k_lanes.err; exit 1; }
cat gpurun_out/r5k_xl_lanes.json
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5k_xl_b64.json 2>> gpurun_out/r5k_lanes.err || { echo B64_FAILED; tail -20 gpurun_out/r5k_lanes.err; exit 1; }
cat gpurun_out/r5k_xl_b64.json
