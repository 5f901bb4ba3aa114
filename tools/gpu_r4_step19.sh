# Round-4 GPU step 19: flash double buffer re-measured in the pipelines after the dispatch-order change
# (decode_ab.py --switch flash_db, prefill tok/s is the figure of interest).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 4"
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch flash_db --values 1,0 --rounds 3 $G \
  > gpurun_out/s19_db_gpt2.jsonl 2> gpurun_out/s19.err || { tail -20 gpurun_out/s19.err; exit 1; }
tail -1 gpurun_out/s19_db_gpt2.jsonl | cut -c1-400
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 2 --warmup 1 --prefill_iters 2"
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch flash_db --values 1,0 --rounds 2 $X \
  > gpurun_out/s19_db_xl.jsonl 2>> gpurun_out/s19.err || { tail -20 gpurun_out/s19.err; exit 1; }
tail -1 gpurun_out/s19_db_xl.jsonl | cut -c1-400
L="--model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 2 --warmup 1 --prefill_iters 2"
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch flash_db --values 1,0 --rounds 2 $L \
  > gpurun_out/s19_db_llama.jsonl 2>> gpurun_out/s19.err || { tail -20 gpurun_out/s19.err; exit 1; }
tail -1 gpurun_out/s19_db_llama.jsonl | cut -c1-400
