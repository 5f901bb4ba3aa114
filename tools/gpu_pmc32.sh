# PMC counters on GPT-2 B=64 decode (decode attention, skinny GEMMs), 2 passes from tools/pmc_decode.txt.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 -i tools/pmc_decode.txt --kernel-trace --output-format csv -d gpurun_out/pmc32 -o run -- python3 bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 4 --warmup 1 --prefill_iters 1 --no_graph > gpurun_out/pmc32.log 2>&1; echo rc=$?
ls -R gpurun_out/pmc32 | head -20
