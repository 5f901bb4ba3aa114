set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/t1.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t1.log
tail -5 gpurun_out/t1.log
timeout -k 10 300 python bench/cifar_quick.py --batches 1,256,4096,65536,262144 > gpurun_out/cq.log 2>&1 && cat gpurun_out/cq.log
