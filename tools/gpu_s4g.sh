export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 500 python -u bench/skinny_sweep.py --m 32,64 --w8 0,1 --shapes gpt2xl,gpt2,llama --iters 10 > gpurun_out/s4g_sweep.jsonl 2> gpurun_out/s4g_sweep.err; echo rc=$?; tail -2 gpurun_out/s4g_sweep.err
