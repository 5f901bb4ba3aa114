# stage-0 v4 with static double-buffer parity / PT: CIFAR tests + flagship bench (x2).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -k "cifar or pipeline or colocated" > gpurun_out/s18_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s18_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > gpurun_out/s18_bench.log 2>&1 && tail -1 gpurun_out/s18_bench.log &&
timeout -k 10 300 python bench.py --steps 40 > gpurun_out/s18_bench2.log 2>&1 && tail -1 gpurun_out/s18_bench2.log &&
timeout -k 10 300 python bench/cifar_quick.py --batches 65536 --iters 20 > gpurun_out/s18_quick.log 2>&1 && tail -3 gpurun_out/s18_quick.log
