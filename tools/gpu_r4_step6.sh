# Round-4 GPU step 6: fused head v2 (balanced tile ranges, image-only prologue wait): tests, isolated
# head probe, decode A/B on GPT-2 B=64 / GPT-2 XL fp8 B=64.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -q --timeout 120 --timeout-method thread -x \
  > gpurun_out/s6_tests.log 2>&1 || { tail -40 gpurun_out/s6_tests.log; exit 1; }
tail -2 gpurun_out/s6_tests.log
timeout -k 10 300 python -u bench/head_probe.py > gpurun_out/s6_head_probe.jsonl 2>&1 || { tail -20 gpurun_out/s6_head_probe.jsonl; exit 1; }
grep "^{" gpurun_out/s6_head_probe.jsonl
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch fused_head --values 0,1 --rounds 3 $G \
  > gpurun_out/s6_ab_head_gpt2.jsonl 2> gpurun_out/s6_ab.err || exit 1
tail -1 gpurun_out/s6_ab_head_gpt2.jsonl | cut -c1-300
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch fused_head --values 0,1 --rounds 2 $X \
  > gpurun_out/s6_ab_head_xl.jsonl 2>> gpurun_out/s6_ab.err || exit 1
tail -1 gpurun_out/s6_ab_head_xl.jsonl | cut -c1-300
