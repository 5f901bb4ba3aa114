mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 200 python bench/cifar_ab.py 65536 2,3 > gpurun_out/ab2.log 2>&1; grep -v amdgpu.ids gpurun_out/ab2.log
timeout -k 10 200 python bench/cifar_ab.py 7 2,3 >> gpurun_out/ab2.log 2>&1; tail -4 gpurun_out/ab2.log
timeout -k 10 200 python bench/cifar_ab.py 262144 2,3 >> gpurun_out/ab2.log 2>&1; tail -2 gpurun_out/ab2.log
