set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gloo_gpu.py > gpurun_out/r5d_gloo.log 2>&1 || { echo GLOO_FAILED; tail -30 gpurun_out/r5d_gloo.log; }
tail -3 gpurun_out/r5d_gloo.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "mx or gpt2_xl_fp8_two_blocks or layernorm_q8 or fp8_gemm or qkv_scatter_prefill_fp8" > gpurun_out/r5d_mx.log 2>&1 || { echo MX_FAILED; tail -40 gpurun_out/r5d_mx.log; exit 1; }
tail -3 gpurun_out/r5d_mx.log
