export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/t5.log 2>&1; tail -1 gpurun_out/t5.log
timeout -k 10 300 python bench.py > gpurun_out/bench5.log 2>&1; tail -1 gpurun_out/bench5.log
timeout -k 10 300 python bench.py --batch 262144 --steps 10 >> gpurun_out/bench5.log 2>&1; tail -1 gpurun_out/bench5.log
