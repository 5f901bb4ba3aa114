# round 3: fc1 A by DMA + fragment split (kernel test, fc1 A/B, pipeline A/B)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "fc1_x3 or split_boundary" --timeout 200 --timeout-method thread -rf -x > gpurun_out/r3_s9_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/probes/cifar_fc1_split_ab.py > gpurun_out/r3_fc1_dma32_ab.jsonl 2> gpurun_out/r3_fc1_dma32_ab.err || exit 1
timeout -k 10 200 python -u bench/probes/cifar_boundary_ab.py > gpurun_out/r3_boundary_ab2.jsonl 2> gpurun_out/r3_boundary_ab2.err || exit 1
