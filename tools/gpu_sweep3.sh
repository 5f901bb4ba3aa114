export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 800 python bench/skinny_sweep.py --m 1,16,32,64 > gpurun_out/skinny_sweep3.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/skinny_sweep3.jsonl; exit $rc
