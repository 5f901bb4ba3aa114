# Round-4 GPU step 12: tail split generalised (partial last column; fp8 256^2 kernel, GPT-2 XL shapes):
# equivalence tests, XL full-width prefill tests, XL and GPT-2 prefill A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -q --timeout 200 \
  --timeout-method thread -x -k "tail_split or qkv_scatter or xl or fp8" > gpurun_out/s12_tests.log 2>&1 || { tail -40 gpurun_out/s12_tests.log; exit 1; }
tail -2 gpurun_out/s12_tests.log
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 2"
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch split_tail --values 0,1 --rounds 2 $X \
  > gpurun_out/s12_ab_split_xl.jsonl 2> gpurun_out/s12_ab.err || exit 1
tail -1 gpurun_out/s12_ab_split_xl.jsonl | cut -c1-300
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 8 --warmup 2 --prefill_iters 3"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch split_tail --values 0,1 --rounds 3 $G \
  > gpurun_out/s12_ab_split_gpt2.jsonl 2>> gpurun_out/s12_ab.err || exit 1
tail -1 gpurun_out/s12_ab_split_gpt2.jsonl | cut -c1-300
