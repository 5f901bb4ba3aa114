#!/bin/bash
# in-process A/B: bf16 skinny row limit 32 (tile path for wide-N heads at M 33-64) vs 64
set -o pipefail
out=gpurun_out/decode_ab.jsonl
: > $out
timeout -k 10 300 python bench/decode_ab.py --switch skinny_max_m --values 32,64 --steps 32 --warmup 4 --prefill_iters 1 >> $out 2>gpurun_out/dab.err &&
timeout -k 10 400 python bench/decode_ab.py --switch skinny_max_m --values 32,64 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1 >> $out 2>>gpurun_out/dab.err
rc=$?; cat $out; exit $rc
