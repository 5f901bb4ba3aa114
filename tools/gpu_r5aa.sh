# Round 5: sanity after a comment-only kernel change (library rebuilt): smoke(), decode GEMM + head GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aa_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r5aa_smoke.log; exit 1; }
tail -1 gpurun_out/r5aa_smoke.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream_gemm_gpu.py tests/test_head_gpu.py tests/test_kernels_gpu.py > gpurun_out/r5aa_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5aa_tests.log; exit 1; }
tail -2 gpurun_out/r5aa_tests.log
