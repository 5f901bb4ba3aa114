export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s4a_tests.log 2>&1 && tail -3 gpurun_out/s4a_tests.log &&
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/s4a_smoke.log 2>&1 && tail -1 gpurun_out/s4a_smoke.log &&
timeout -k 10 200 python bench.py > gpurun_out/s4a_bench.log 2>&1 && tail -1 gpurun_out/s4a_bench.log &&
timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 > gpurun_out/s4a_llama_b1.log 2>&1 && tail -1 gpurun_out/s4a_llama_b1.log
