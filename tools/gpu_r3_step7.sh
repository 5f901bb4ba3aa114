# round 3: split boundary encoding (kernel + pipeline tests, A/B, bench line)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -q --timeout 300 --timeout-method thread -rf -x > gpurun_out/r3_s7_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/probes/cifar_boundary_ab.py > gpurun_out/r3_boundary_ab.jsonl 2> gpurun_out/r3_boundary_ab.err || exit 1
timeout -k 10 300 python -u bench.py --no_extra > gpurun_out/r3_s7_bench.log 2>&1 || exit 1
