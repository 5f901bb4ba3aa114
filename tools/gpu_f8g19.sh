# fp8 256^2 GEMM: fp8 tests, fp8 GEMM bench, fp8 prefill benches (GPT-2 XL, Llama-3 8B).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8" > gpurun_out/f19_tests.log 2>&1; rc=$?; tail -2 gpurun_out/f19_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gemm_fp8_bench.py > gpurun_out/f19_gemm.jsonl 2>&1 && cat gpurun_out/f19_gemm.jsonl &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 16 > gpurun_out/f19_xl.log 2>&1 && tail -1 gpurun_out/f19_xl.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --dtype fp8 --batch 32 --prompt 512 --steps 16 > gpurun_out/f19_llama.log 2>&1 && tail -1 gpurun_out/f19_llama.log
