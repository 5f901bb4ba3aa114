export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s4i_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s4i_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/cifar_ab.py 65536 3@24,3@28,4@24,4@28,4@32 2>&1 | grep -v amdgpu.ids
