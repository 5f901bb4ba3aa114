# Fused QKV prefill attention: transformer tests + GPT-2 bench + kernel profile.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f8_tests.log 2>&1; rc=$?; tail -3 gpurun_out/f8_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 > gpurun_out/f8_gpt2.log 2>&1 && tail -1 gpurun_out/f8_gpt2.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f8_prof -o run -- python3 bench/gpt_bench.py --batch 64 --prompt 512 --steps 4 --prefill_iters 3 > gpurun_out/f8_prof.log 2>&1
