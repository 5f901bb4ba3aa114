# round 3: forced stream GEMM vs the measured plan on the three decode configs (in-process A/B)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch stream --values 1,2 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_stream_forced_gpt2xl.jsonl 2> gpurun_out/r3_stream_forced_gpt2xl.err || exit 1
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch stream --values 1,2 --rounds 2 --model gpt2 --stages 4 --batch 64 --prompt 512 --dtype bf16 --steps 32 --warmup 2 --prefill_iters 1 > gpurun_out/r3_stream_forced_gpt2.jsonl 2> gpurun_out/r3_stream_forced_gpt2.err || exit 1
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch stream --values 1,2 --rounds 2 --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_stream_forced_llama.jsonl 2> gpurun_out/r3_stream_forced_llama.err || exit 1
