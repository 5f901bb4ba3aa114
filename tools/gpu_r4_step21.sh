# Round-4 GPU step 21: flash prefill with Q fragments in LDS (128 VGPRs, 4 workgroups per CU, one K/V buffer):
# attention tests with the variant forced, then GPT-2 / GPT-2 XL prefill A/B in one process.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DNN_FLASH_QL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_kv8_gpu.py tests/test_transformer_gpu.py -k "flash or qkv or prefill" > gpurun_out/s21_tests.log 2>&1 || { tail -30 gpurun_out/s21_tests.log; exit 1; }
tail -1 gpurun_out/s21_tests.log
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 4"
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch flash_ql --values 0,1 --rounds 3 $G \
  > gpurun_out/s21_ql_gpt2.jsonl 2> gpurun_out/s21.err || { tail -20 gpurun_out/s21.err; exit 1; }
tail -1 gpurun_out/s21_ql_gpt2.jsonl | cut -c1-400
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 2 --warmup 1 --prefill_iters 2"
timeout -k 10 500 python -u bench/probes/decode_ab.py --switch flash_ql --values 0,1 --rounds 2 $X \
  > gpurun_out/s21_ql_xl.jsonl 2>> gpurun_out/s21.err || { tail -20 gpurun_out/s21.err; exit 1; }
tail -1 gpurun_out/s21_ql_xl.jsonl | cut -c1-400
