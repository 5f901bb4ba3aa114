# decode attention: 16 rows in flight per thread for MHA hd 64 (GPT-2, GPT-2 XL).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode" > gpurun_out/u15_tests.log 2>&1; rc=$?; tail -2 gpurun_out/u15_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/u15_gpt2.log 2>&1 && tail -1 gpurun_out/u15_gpt2.log &&
timeout -k 10 400 python bench/gpt_bench.py --model gpt2-xl --stages 8 --dtype fp8 --batch 64 --prompt 512 --steps 32 > gpurun_out/u15_xl.log 2>&1 && tail -1 gpurun_out/u15_xl.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u15_prof -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 8 --prefill_iters 1 > gpurun_out/u15_prof.log 2>&1
