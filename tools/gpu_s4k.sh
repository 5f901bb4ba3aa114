export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stage0 or cifar" > gpurun_out/s4k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s4k_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/cifar_ab.py 65536 3@28,4@24,4@28,4@32 2>&1 | grep -v amdgpu.ids | grep ms_median
