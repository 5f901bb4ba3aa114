export PYTHONPATH=$PWD
timeout -k 10 120 python bench/cifar_stamps.py 65536 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python bench/cifar_ab.py 65536 2,3 2>&1 | grep -v amdgpu.ids
