# Round-4 GPU step 9: prefill tail split (256^2 + 256x128 launches for GPT-2's 768-wide O / c_proj):
# equivalence tests, isolated GEMM arms (auto = split vs forced 256^2), GPT-2 prefill A/B in the pipeline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -x \
  -k "tail_split or 256" > gpurun_out/s9_tests.log 2>&1 || { tail -40 gpurun_out/s9_tests.log; exit 1; }
tail -2 gpurun_out/s9_tests.log
timeout -k 10 200 python -u bench/gemm_bench.py --tiles 0,256 --rounds 3 --inplace --shapes 32768x768x768,32768x768x3072 \
  > gpurun_out/s9_gemm_split.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench/gemm_bench.py --tiles 0,256 --rounds 3 --shapes 32768x768x768,32768x768x3072 \
  >> gpurun_out/s9_gemm_split.jsonl 2>&1 || exit 1
grep "^{" gpurun_out/s9_gemm_split.jsonl | cut -c1-250
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 8 --warmup 2 --prefill_iters 3"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch split_tail --values 0,1 --rounds 3 $G \
  > gpurun_out/s9_ab_split_gpt2.jsonl 2> gpurun_out/s9_ab.err || exit 1
tail -1 gpurun_out/s9_ab_split_gpt2.jsonl | cut -c1-300
