# round 3: stream GEMM plan v2 — tests, A/B, decode A/B + kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_stream_gemm_gpu.py tests/test_transformer_gpu.py tests/test_kv8_gpu.py -q --timeout 200 --timeout-method thread -rf -k "stream or full_width or fp8_stage_runs or llama_tiny_decode_kv8" > gpurun_out/r3_tests5.log 2>&1
timeout -k 10 300 python -u bench/stream_gemm_ab.py --m 32 --shapes llama > gpurun_out/r3_stream_ab2_llama.jsonl 2>&1 || exit 1
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch stream --values 0,1 --rounds 2 --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_stream_decode_ab2.jsonl 2> gpurun_out/r3_stream_decode_ab2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_llama32b -o run -- python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 8 --warmup 1 --prefill_iters 1 > gpurun_out/prof_llama32b.log 2>&1 || exit 1
