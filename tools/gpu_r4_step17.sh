# Round-4 GPU step 17: flash prefill A/B in one process (bench/probes/flash_bench.py): longest query blocks dispatched first.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench/probes/flash_bench.py > gpurun_out/s17_flash_lpt_ab.jsonl 2> gpurun_out/s17.err || { tail -20 gpurun_out/s17.err; exit 1; }
cat gpurun_out/s17_flash_lpt_ab.jsonl
