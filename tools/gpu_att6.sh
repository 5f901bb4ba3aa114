# Flash-attention VALU trims + decode split A/B (GPT-2 B=64, Llama B=32).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or flash or transformer or prefill or decode" > gpurun_out/a6_tests.log 2>&1; rc=$?; tail -3 gpurun_out/a6_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/a6_gpt2.log 2>&1 && tail -1 gpurun_out/a6_gpt2.log &&
DNN_DECODE_SPLITS=1 timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/a6_gpt2_s1.log 2>&1 && tail -1 gpurun_out/a6_gpt2_s1.log &&
DNN_DECODE_SPLITS=4 timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/a6_gpt2_s4.log 2>&1 && tail -1 gpurun_out/a6_gpt2_s4.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/a6_llama.log 2>&1 && tail -1 gpurun_out/a6_llama.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a6_prof -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 4 --prefill_iters 3 > gpurun_out/a6_prof.log 2>&1
