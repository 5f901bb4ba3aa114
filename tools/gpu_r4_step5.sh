# Round-4 GPU step 5: the fused decode head (gemm_head.h) — its tests, the decode A/B
# (fused_head 0/1) on GPT-2 B=64 and GPT-2 XL fp8 B=64, and a kernel table of the GPT-2 step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -v --timeout 120 --timeout-method thread -x \
  > gpurun_out/s5_tests.log 2>&1 || { tail -40 gpurun_out/s5_tests.log; exit 1; }
tail -3 gpurun_out/s5_tests.log
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch fused_head --values 0,1 --rounds 3 $G \
  > gpurun_out/s5_ab_head_gpt2.jsonl 2> gpurun_out/s5_ab.err || exit 1
tail -1 gpurun_out/s5_ab_head_gpt2.jsonl | cut -c1-300
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch fused_head --values 0,1 --rounds 2 $X \
  > gpurun_out/s5_ab_head_xl.jsonl 2>> gpurun_out/s5_ab.err || exit 1
tail -1 gpurun_out/s5_ab_head_xl.jsonl | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run -- python3 bench/gpt_bench.py $G > gpurun_out/prof_s5.log 2>&1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/prof_s5 > gpurun_out/s5_gpt2_kernels.md
rm -rf gpurun_out/prof_s5
grep -E "head|argmax|skinny" gpurun_out/s5_gpt2_kernels.md | cut -c1-200
