# Single-pass decode attention: transformer tests + decode benches.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/d9_tests.log 2>&1; rc=$?; tail -3 gpurun_out/d9_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/d9_gpt2.log 2>&1 && tail -1 gpurun_out/d9_gpt2.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/d9_llama32.log 2>&1 && tail -1 gpurun_out/d9_llama32.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/d9_llama1.log 2>&1 && tail -1 gpurun_out/d9_llama1.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/d9_xl.log 2>&1 && tail -1 gpurun_out/d9_xl.log
