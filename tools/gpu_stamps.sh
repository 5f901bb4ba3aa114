export PYTHONPATH=$PWD
timeout -k 10 200 python bench/cifar_stamps.py 65536 ${PTS:-16,20,24,28,32} 2>&1 | grep -v amdgpu.ids
