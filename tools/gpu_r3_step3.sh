# round 3: stream GEMM eligibility, full-width fp8 test, decode benches
set -o pipefail
timeout -k 10 200 python -u bench/probes/fp8_prefill_probe.py > gpurun_out/r3_fp8_probe2.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_stream_gemm_gpu.py tests/test_kv8_gpu.py tests/test_transformer_gpu.py -q --timeout 200 --timeout-method thread -rf -k "stream or llama_tiny_decode_kv8 or full_width" > gpurun_out/r3_tests3.log 2>&1
for a in "--model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16" "--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8" "--model gpt2 --stages 4 --batch 64 --prompt 512 --dtype bf16"; do
  timeout -k 10 300 python -u bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1 $a >> gpurun_out/r3_decode_benches.jsonl 2>> gpurun_out/r3_decode_benches.err || exit 1
done
