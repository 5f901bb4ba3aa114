export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python bench/skinny_sweep.py --m 1,32 > gpurun_out/skinny_sweep.jsonl 2>&1; rc=$?; cat gpurun_out/skinny_sweep.jsonl | cut -c1-400; exit $rc
