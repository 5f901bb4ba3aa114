# Round 5: one-shot decode GEMM anatomy (launch alone, no reduction).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench/probes/oneshot_anatomy.py > gpurun_out/r5n_oneshot_anatomy.jsonl 2> gpurun_out/r5n_anat.err || { echo ANAT_FAILED; tail -20 gpurun_out/r5n_anat.err; exit 1; }
cat gpurun_out/r5n_oneshot_anatomy.jsonl
