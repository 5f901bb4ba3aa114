# Round-4 GPU step 14: fp8 tail split by tail width on the GPT-2 XL prefill (mask 1 bf16 only, 5 + fp8 tails
# >= 128 columns, 3 + every fp8 tail).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 2"
timeout -k 10 600 python -u bench/probes/decode_ab.py --switch split_tail --values 1,5,3 --rounds 3 $X \
  > gpurun_out/s14_ab_split_xl.jsonl 2> gpurun_out/s14_ab.err || exit 1
tail -1 gpurun_out/s14_ab_split_xl.jsonl | cut -c1-400
