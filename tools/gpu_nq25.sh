# fused normalise+quantise for fp8 prefill: fp8/stage tests, XL + Llama fp8 benches.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8 or q8 or stage or w8" > gpurun_out/n25_tests.log 2>&1; rc=$?; tail -2 gpurun_out/n25_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 8 > gpurun_out/n25_xl.log 2>&1 && tail -1 gpurun_out/n25_xl.log | cut -c1-600 &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --dtype fp8 --batch 32 --prompt 512 --steps 8 > gpurun_out/n25_llama.log 2>&1 && tail -1 gpurun_out/n25_llama.log | cut -c1-600
