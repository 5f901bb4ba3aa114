# Round verification on one MI355X: GPU tests, smoke, the driver's bench line, and a
# rocprofv3 kernel table of the Llama-3 8B B=32 decode (gpurun_out/v_*).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/v_tests.log 2>&1
rc=$?; tail -4 gpurun_out/v_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/v_smoke.log | cut -c1-120
timeout -k 10 600 python -u bench.py > gpurun_out/v_bench.log 2>&1 || exit 1
tail -1 gpurun_out/v_bench.log > gpurun_out/v_bench.json; cut -c1-300 gpurun_out/v_bench.json
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v -o run -- python3 $L > gpurun_out/prof_v.log 2>&1 &&
python3 tools/rocprof_summary.py gpurun_out/prof_v > gpurun_out/v_llama_b32_kernels.md; rc=$?
rm -rf gpurun_out/prof_v; exit $rc
