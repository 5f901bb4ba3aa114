# round 3: decode A/B of the stream GEMM + kernel trace of Llama-3 8B B=32 decode
set -o pipefail
cd /root/repo
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch stream --values 0,1,2 --rounds 2 --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_stream_decode_ab.jsonl 2> gpurun_out/r3_stream_decode_ab.err || exit 1
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch stream --values 0,1 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 >> gpurun_out/r3_stream_decode_ab.jsonl 2>> gpurun_out/r3_stream_decode_ab.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llama32 -o run -- python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 8 --warmup 1 --prefill_iters 1 > gpurun_out/prof_llama32.log 2>&1 || exit 1
