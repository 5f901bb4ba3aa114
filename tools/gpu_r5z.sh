# Round 5: race screen over pinned one-shot configurations with and without the one-workgroup-per-CU LDS floor.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u bench/probes/epi_race_screen.py --iters 300 --cases ln_gelu_2304x768_forced,ln_gelu_2304x768_pin111,ln_gelu_2304x768_pin211,nofloor_ln_gelu_2304x768_pin111,nofloor_ln_gelu_2304x768_pin211 > gpurun_out/r5z_race.jsonl 2> gpurun_out/r5z_race.err || { echo RACE_FAILED; tail -20 gpurun_out/r5z_race.err; exit 1; }
cat gpurun_out/r5z_race.jsonl
