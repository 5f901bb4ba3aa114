mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_transformer_gpu.py -x -q -k "decode or stage" > gpurun_out/tests4.log 2>&1; rc=$?; tail -2 gpurun_out/tests4.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 32 > gpurun_out/llama_b32.log 2>&1 && tail -1 gpurun_out/llama_b32.log &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof1 -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/lprof1.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof32 -o run -- python3 bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 8 --warmup 2 --prefill_iters 1 --no_graph > gpurun_out/lprof32.log 2>&1; echo rc=$?
