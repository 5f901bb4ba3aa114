# Fragment-order decode weights: full GPU tests, then decode benches (Llama B=32/B=1 bf16+fp8, GPT-2, XL).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s14_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s14_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/s14_llama32.log 2>&1 && tail -1 gpurun_out/s14_llama32.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --dtype fp8 > gpurun_out/s14_llama32f8.log 2>&1 && tail -1 gpurun_out/s14_llama32f8.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/s14_llama1.log 2>&1 && tail -1 gpurun_out/s14_llama1.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 --dtype fp8 > gpurun_out/s14_llama1f8.log 2>&1 && tail -1 gpurun_out/s14_llama1f8.log &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/s14_gpt2.log 2>&1 && tail -1 gpurun_out/s14_gpt2.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/s14_xl.log 2>&1 && tail -1 gpurun_out/s14_xl.log
