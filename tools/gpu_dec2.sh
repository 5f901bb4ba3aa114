export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/tests8.log 2>&1; rc=$?; tail -2 gpurun_out/tests8.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/gpt_b64.log 2>&1 && tail -1 gpurun_out/gpt_b64.log | cut -c1-200 &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 > gpurun_out/llama_b32.log 2>&1 && tail -1 gpurun_out/llama_b32.log | cut -c1-200 &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/llama_b1.log 2>&1 && tail -1 gpurun_out/llama_b1.log | cut -c1-200 &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/xl_fp8_b64.log 2>&1 && tail -1 gpurun_out/xl_fp8_b64.log | cut -c1-200 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof1c -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/lprof1c.log 2>&1; echo rc=$?
