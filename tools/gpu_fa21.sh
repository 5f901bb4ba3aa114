# flash prefill with register double-buffered K/V: attention tests, GPT-2 / Llama prefill, kernel times.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or stage or qkv" > gpurun_out/a21_tests.log 2>&1; rc=$?; tail -2 gpurun_out/a21_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 8 > gpurun_out/a21_gpt2.log 2>&1 && tail -1 gpurun_out/a21_gpt2.log &&
timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 8 > gpurun_out/a21_llama.log 2>&1 && tail -1 gpurun_out/a21_llama.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a21_prof -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 2 --prefill_iters 3 > gpurun_out/a21_prof.log 2>&1
