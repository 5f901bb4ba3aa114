# round 3: folded split-K combine (tests + decode A/B), then the full verification
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stream_gemm_gpu.py -q --timeout 200 --timeout-method thread -rf -x > gpurun_out/r3_stream_tests6.log 2>&1 || exit 1
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch stream_fold --values 0,1 --rounds 2 --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_fold_decode_ab.jsonl 2> gpurun_out/r3_fold_decode_ab.err || exit 1
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch decode_splits --values 0,1,2 --rounds 1 --model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r3_splits_decode_ab.jsonl 2> gpurun_out/r3_splits_decode_ab.err || exit 1
bash tools/gpu_r3_verify.sh
