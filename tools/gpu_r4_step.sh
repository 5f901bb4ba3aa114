# Round-4 GPU step: changed tests, the gloo_gpu pre-post A/B, the one-shot GEMM sweep, the bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u bench/oneshot_sweep.py > gpurun_out/s1_oneshot.jsonl 2> gpurun_out/s1_oneshot.err || exit 1
cut -c1-300 gpurun_out/s1_oneshot.jsonl
timeout -k 10 900 python -u -m pytest tests/test_native_comm_gpu.py tests/test_kv8_gpu.py tests/test_gloo_gpu.py \
  tests/test_transformer_gpu.py tests/test_stream_gemm_gpu.py -k "native or kv8 or gloo or split or full_width or oneshot" \
  -m gpu -q \
  --timeout 300 --timeout-method thread -rfs > gpurun_out/s1_tests.log 2>&1
rc=$?; tail -6 gpurun_out/s1_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench/gpt_bench.py --gpus 4 --gloo_gpu --model gpt2-tiny --stages 4 --batch 8 --prompt 64 \
  --steps 16 --warmup 2 --prefill_iters 1 --microbatches 8 --prepost_ab 3 > gpurun_out/s1_prepost_ab.log 2>&1 || exit 1
grep '^{' gpurun_out/s1_prepost_ab.log | tail -1 > gpurun_out/s1_prepost_ab.json; cut -c1-600 gpurun_out/s1_prepost_ab.json
timeout -k 10 600 python -u bench.py > gpurun_out/s1_bench.log 2>&1 || exit 1
tail -1 gpurun_out/s1_bench.log > gpurun_out/s1_bench.json; cut -c1-400 gpurun_out/s1_bench.json
