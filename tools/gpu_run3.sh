set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/test_transformer_gpu.py -x -q > gpurun_out/t3.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t3.log
tail -30 gpurun_out/t3.log
