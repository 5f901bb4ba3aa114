mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python bench/cifar_ab.py 65536 1,2 > gpurun_out/ab1.log 2>&1; cat gpurun_out/ab1.log | grep -v amdgpu.ids
timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -q -x -k cifar >> gpurun_out/ab1.log 2>&1; tail -2 gpurun_out/ab1.log
timeout -k 10 200 python bench.py >> gpurun_out/ab1.log 2>&1; tail -1 gpurun_out/ab1.log
