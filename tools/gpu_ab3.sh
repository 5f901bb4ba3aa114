mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python bench/cifar_ab.py 65536 2,3 > gpurun_out/ab3.log 2>&1; grep -v amdgpu.ids gpurun_out/ab3.log
timeout -k 10 200 python bench/cifar_ab.py 5 2,3 >> gpurun_out/ab3.log 2>&1; tail -2 gpurun_out/ab3.log
timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -q -x -k cifar >> gpurun_out/ab3.log 2>&1; tail -1 gpurun_out/ab3.log
