# round 3: full verification (GPU tests, smoke, driver bench line) + GPT-2 XL fp8 decode kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > gpurun_out/r3_v_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_v_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r3_v_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gpt2xl64 -o run -- python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 8 --warmup 1 --prefill_iters 1 > gpurun_out/prof_gpt2xl64.log 2>&1 || exit 1
