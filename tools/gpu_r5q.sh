set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python bench/probes/epi_pre_diff.py > gpurun_out/r5q_diff.jsonl 2> gpurun_out/r5q.err || { echo FAILED; tail -20 gpurun_out/r5q.err; exit 1; }
cat gpurun_out/r5q_diff.jsonl
