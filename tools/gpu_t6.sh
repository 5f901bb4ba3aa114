export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/ -m gpu -q -x > gpurun_out/t6.log 2>&1; tail -3 gpurun_out/t6.log
timeout -k 10 200 python __graft_entry__.py smoke 2>&1 | tail -1
