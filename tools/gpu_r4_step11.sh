# Round-4 GPU step 11: tail split of the QKV scatter GEMM — tests, GPT-2 prefill A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kernels_gpu.py -q --timeout 120 \
  --timeout-method thread -x -k "qkv_scatter or tail_split or gpt2" > gpurun_out/s11_tests.log 2>&1 || { tail -40 gpurun_out/s11_tests.log; exit 1; }
tail -2 gpurun_out/s11_tests.log
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 8 --warmup 2 --prefill_iters 3"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch split_tail --values 0,1 --rounds 3 $G \
  > gpurun_out/s11_ab_split_gpt2.jsonl 2> gpurun_out/s11_ab.err || exit 1
tail -1 gpurun_out/s11_ab_split_gpt2.jsonl | cut -c1-300
