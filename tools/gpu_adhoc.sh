# Ad-hoc GPU batch: each argument is one shell step, run under its own 900 s
# timeout, stopping at the first failure (no retries); outputs under
# gpurun_out/.  Keeps one-off experiment lists out of tools/ (tools/gpu_runs.md
# records which profiles/ file came from which step list).
#   gpurun --timeout 1200 -- 'bash tools/gpu_adhoc.sh "step 1" "step 2" ...'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for step in "$@"; do
  k=$((k + 1))
  echo "== [$k] $step"
  timeout -k 10 900 bash -c "$step" || { echo "STEP_FAILED rc=$? [$k]"; exit 1; }
done
