# round 3 session 2, step 5: full GPU tests + smoke + driver bench line; Llama-3 8B B=32 decode kernel table
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/s5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/s5_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/s5_smoke.log | cut -c1-120
timeout -k 10 600 python -u bench.py > gpurun_out/s5_bench.log 2>&1 || exit 1
tail -1 gpurun_out/s5_bench.log > gpurun_out/s5_bench.json; cut -c1-300 gpurun_out/s5_bench.json
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run -- python3 $L > gpurun_out/prof_s5.log 2>&1 &&
python3 tools/rocprof_summary.py gpurun_out/prof_s5 > gpurun_out/s5_llama_b32_kernels.md; rc=$?
rm -rf gpurun_out/prof_s5; exit $rc
