# Kernel breakdown of the fp8 prefill (GPT-2 XL 8-stage, B=64 x 512).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xl24 -o run -- python3 bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 2 --prefill_iters 2 > gpurun_out/xl24.log 2>&1
