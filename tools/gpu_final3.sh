# Round-end verification: full GPU tests, smoke, flagship bench (+ rocprof kernel table), GPT-2 bench via bench.py,
# decode/prefill benches for every BASELINE transformer config.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fin3_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin3_smoke.log 2>&1 && tail -1 gpurun_out/fin3_smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/fin3_bench.log 2>&1 && tail -1 gpurun_out/fin3_bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin3_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/fin3_prof.log 2>&1 &&
timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/fin3_gpt2.log 2>&1 && tail -1 gpurun_out/fin3_gpt2.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/fin3_llama32.log 2>&1 && tail -1 gpurun_out/fin3_llama32.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --dtype fp8 > gpurun_out/fin3_llama32f8.log 2>&1 && tail -1 gpurun_out/fin3_llama32f8.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/fin3_llama1.log 2>&1 && tail -1 gpurun_out/fin3_llama1.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 --dtype fp8 > gpurun_out/fin3_llama1f8.log 2>&1 && tail -1 gpurun_out/fin3_llama1f8.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/fin3_xl.log 2>&1 && tail -1 gpurun_out/fin3_xl.log
