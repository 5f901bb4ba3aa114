# Round 5: GPT-2 4-stage decode kernel table at B=64 (final library), then the large-batch capacity points
# (B = 512 / 1024, bf16 and fp8 KV; tools/gpu_r5p.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
G="bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run -- python3 $G > gpurun_out/prof_v1.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_v1.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof_v1 > gpurun_out/r5v_gpt2_b64_decode_kernels.md
rm -rf gpurun_out/prof_v1
head -14 gpurun_out/r5v_gpt2_b64_decode_kernels.md
bash tools/gpu_r5p.sh
