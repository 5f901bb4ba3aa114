# Kernel-time breakdown of the transformer prefill paths (GPT-2 small 4-stage, Llama-3 8B 8-stage).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_gpt2 -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 2 --prefill_iters 5 > gpurun_out/pp_gpt2.log 2>&1 && tail -1 gpurun_out/pp_gpt2.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_llama -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 2 --prefill_iters 3 > gpurun_out/pp_llama.log 2>&1 && tail -1 gpurun_out/pp_llama.log
