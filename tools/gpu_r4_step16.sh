# Round-4 GPU step 16: NaN-propagating max (v_maximum3_f32, no IEEE canonicalisation) in the flash softmax and
# the CIFAR pools — attention/CIFAR tests, GPT-2 prefill kernel table, bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_kv8_gpu.py tests/test_transformer_gpu.py -k "flash or cifar or qkv or attn" > gpurun_out/s16_tests.log 2>&1 || { tail -30 gpurun_out/s16_tests.log; exit 1; }
tail -2 gpurun_out/s16_tests.log
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run -- python3 $G > gpurun_out/prof16.log 2>&1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/prof16 > gpurun_out/s16_prefill_kernels.md
rm -rf gpurun_out/prof16
grep "flash_attn" gpurun_out/s16_prefill_kernels.md | cut -c1-160
timeout -k 10 600 python bench.py > gpurun_out/s16_bench.log 2>&1 || { tail -20 gpurun_out/s16_bench.log; exit 1; }
tail -1 gpurun_out/s16_bench.log | cut -c1-900
