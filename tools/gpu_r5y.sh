# Round 5: race screen with mismatch detail (column tiles, rows, counts); skinny and planned one-shot arms of the same shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u bench/probes/epi_race_screen.py --iters 300 --cases ln_gelu_2304x768_forced,ln_gelu_2304x768_skinny,ln_gelu_2304x768_planned,ln_gelu_3072x768_forced > gpurun_out/r5y_race.jsonl 2> gpurun_out/r5y_race.err || { echo RACE_FAILED; tail -20 gpurun_out/r5y_race.err; exit 1; }
cat gpurun_out/r5y_race.jsonl
