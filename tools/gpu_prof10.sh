# Decode-attention kernel times after the single-pass rewrite (Llama B=32, GPT-2 B=64).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p10_llama -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 8 --prefill_iters 1 > gpurun_out/p10_llama.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p10_gpt2 -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 8 --prefill_iters 1 > gpurun_out/p10_gpt2.log 2>&1
