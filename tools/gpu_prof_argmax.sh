set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_amx -o run -- python3 $L > gpurun_out/prof_amx.log 2>&1 &&
python3 tools/rocprof_gaps.py gpurun_out/prof_amx > gpurun_out/amx_gaps.md
rc=$?; rm -rf gpurun_out/prof_amx; head -14 gpurun_out/amx_gaps.md; exit $rc
