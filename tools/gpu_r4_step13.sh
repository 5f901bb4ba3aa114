# Round-4 GPU step 13: tail-split tests with the fp8 bit opt-in.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -q --timeout 200 \
  --timeout-method thread -x -k "tail_split or qkv_scatter or fp8" > gpurun_out/s13_tests.log 2>&1 || { tail -40 gpurun_out/s13_tests.log; exit 1; }
tail -2 gpurun_out/s13_tests.log
