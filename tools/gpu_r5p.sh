# Round 5: GPT-2 4-stage decode at large batch (HBM capacity points): B = 512 / 1024, bf16 and fp8 KV.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for B in 512 1024; do
  timeout -k 10 300 python bench/gpt_bench.py --batch $B --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5p_b$B.json 2> gpurun_out/r5p_b$B.err || { echo B${B}_FAILED; tail -20 gpurun_out/r5p_b$B.err; exit 1; }
  cat gpurun_out/r5p_b$B.json
  timeout -k 10 300 python bench/gpt_bench.py --batch $B --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 --kv fp8 > gpurun_out/r5p_b${B}_kv8.json 2> gpurun_out/r5p_b${B}_kv8.err || { echo B${B}KV8_FAILED; tail -20 gpurun_out/r5p_b${B}_kv8.err; exit 1; }
  cat gpurun_out/r5p_b${B}_kv8.json
done
