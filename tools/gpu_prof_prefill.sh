#!/bin/bash
# GPT-2 4-stage prefill (B=64, T=512) per-call kernel sequence of one layer
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp -o run -- python3 bench/gpt_bench.py --steps 2 --warmup 1 --prefill_iters 2 > gpurun_out/pp.log 2>&1
rc=$?
python3 tools/rocprof_seq.py gpurun_out/pp --marker flash_attn --occurrence 14 --before 3 --count 16 > gpurun_out/prefill_seq.md
rm -rf gpurun_out/pp
exit $rc
