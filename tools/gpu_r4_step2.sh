# Round-4 GPU step 2: full GPU tests, one-shot decode A/B in the pipeline, 256x128 prefill tiles,
# the gloo_gpu pre-post A/B with asynchronous host-staged sends, the CIFAR overlap probe.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs -x \
  > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -8 gpurun_out/s2_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 3"
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 2 $G \
  > gpurun_out/s2_ab_oneshot_gpt2.jsonl 2> gpurun_out/s2_ab.err || exit 1
tail -1 gpurun_out/s2_ab_oneshot_gpt2.jsonl
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 2 $X \
  > gpurun_out/s2_ab_oneshot_xl.jsonl 2>> gpurun_out/s2_ab.err || exit 1
tail -1 gpurun_out/s2_ab_oneshot_xl.jsonl
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch gemm_tile --values 256,0 --rounds 2 $G \
  > gpurun_out/s2_ab_tile_gpt2.jsonl 2>> gpurun_out/s2_ab.err || exit 1
tail -1 gpurun_out/s2_ab_tile_gpt2.jsonl
timeout -k 10 200 python -u bench/gemm_bench.py --tiles 256,255 --rounds 2 \
  --shapes 32768x768x768,32768x768x3072,32768x2304x768,32768x3072x768,16384x4096x4096 > gpurun_out/s2_gemm_tiles.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench/gemm_bench.py --tiles 256,255 --rounds 2 --act gelu --shapes 32768x3072x768,32768x2304x768 \
  > gpurun_out/s2_gemm_tiles_gelu.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench/gemm_bench.py --tiles 256,255 --rounds 2 --residual --shapes 32768x768x768,32768x768x3072 \
  > gpurun_out/s2_gemm_tiles_res.jsonl 2>&1 || exit 1
cat gpurun_out/s2_gemm_tiles*.jsonl | cut -c1-200
timeout -k 10 300 python -u bench/gpt_bench.py --gpus 4 --gloo_gpu --model gpt2-tiny --stages 4 --batch 8 --prompt 64 \
  --steps 16 --warmup 2 --prefill_iters 1 --microbatches 8 --prepost_ab 3 > gpurun_out/s2_prepost_ab.log 2>&1 || exit 1
grep '^{' gpurun_out/s2_prepost_ab.log | tail -1 > gpurun_out/s2_prepost_ab.json; cut -c1-300 gpurun_out/s2_prepost_ab.json
timeout -k 10 200 python -u bench/probes/cifar_overlap_ab.py > gpurun_out/s2_cifar_overlap.jsonl 2>&1 || exit 1
cat gpurun_out/s2_cifar_overlap.jsonl | cut -c1-600
