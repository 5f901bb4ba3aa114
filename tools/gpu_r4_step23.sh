# Round-4 GPU step 23: fused decode head, load-group size A/B in one process (bench/head_probe.py, temporary DNN_HEAD_GS).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench/head_probe.py > gpurun_out/s23_head_gs.jsonl 2> gpurun_out/s23.err || { tail -20 gpurun_out/s23.err; exit 1; }
cat gpurun_out/s23_head_gs.jsonl
