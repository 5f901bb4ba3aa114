# One parameterised GPU runner (replaces the one-off tools/gpu_r4_*/gpu_r5*.sh
# scripts, which stay in the git history; tools/gpu_runs.md maps every
# profiles/ file to the command that produced it).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh TAG STEP [STEP ...]'
#
# STEP is one of
#   tests            pytest -m gpu (whole suite, thread timeouts)
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (the driver's default line)
#   kernels:CFG      rocprofv3 --kernel-trace --stats of bench/gpt_bench.py CFG
#                    (gpt2 | gpt2xl | llama), summarised by tools/rocprof_summary.py
#   gaps:CFG         the same trace's inter-kernel gaps (tools/rocprof_gaps.py)
#   pmc:CFG          two rocprofv3 --pmc passes (tools/gpu_pmc.sh), tools/pmc_summary.py
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (ARGS with ',' for spaces), stdout to gpurun_out/TAG_<name>_<k>.jsonl
#                    (k counts the py steps of the call)
# Every GPU step runs under its own timeout and the script stops at the first
# failure (no retries).  Outputs: gpurun_out/TAG_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1
shift
mkdir -p gpurun_out
O=gpurun_out/$TAG
pyk=0

cfg_args() {
  case $1 in
    gpt2) echo "--model gpt2 --stages 4 --batch 64 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1" ;;
    gpt2xl) echo "--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1" ;;
    llama) echo "--model llama3-8b --stages 8 --batch 32 --prompt 512 --dtype bf16 --steps 16 --warmup 2 --prefill_iters 1" ;;
    *) echo "unknown config $1" >&2; return 1 ;;
  esac
}

for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf \
        > ${O}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 ${O}_tests.log; exit 1; }
      tail -3 ${O}_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 \
        || { echo SMOKE_FAILED; tail -20 ${O}_smoke.log; exit 1; }
      tail -1 ${O}_smoke.log | cut -c1-300 ;;
    bench)
      timeout -k 10 600 python bench.py > ${O}_bench.json 2> ${O}_bench.err \
        || { echo BENCH_FAILED; tail -20 ${O}_bench.err; exit 1; }
      cut -c1-600 ${O}_bench.json ;;
    kernels:*|gaps:*)
      c=${step#*:}
      a=$(cfg_args $c) || exit 1
      d=${O}_trace_$c
      if [ ! -d $d ]; then
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
          python3 bench/gpt_bench.py $a > ${O}_trace_$c.log 2>&1 || { echo TRACE_FAILED; tail -20 ${O}_trace_$c.log; exit 1; }
      fi
      if [ ${step%%:*} = kernels ]; then
        python tools/rocprof_summary.py $d > ${O}_${c}_kernels.md && head -30 ${O}_${c}_kernels.md
      else
        python tools/rocprof_gaps.py $d > ${O}_${c}_gaps.md && head -30 ${O}_${c}_gaps.md
      fi ;;
    pmc:*)
      c=${step#*:}
      a=$(cfg_args $c) || exit 1
      bash tools/gpu_pmc.sh ${O}_pmc_$c bench/gpt_bench.py $a || { echo PMC_FAILED; tail -20 ${O}_pmc_$c/p*.log; exit 1; }
      python tools/pmc_summary.py --min_grid 1 --top 16 ${O}_pmc_$c > ${O}_pmc_${c}.md && head -40 ${O}_pmc_${c}.md ;;
    py:*)
      spec=${step#py:}
      script=${spec%%:*}
      args=""
      [ "$spec" != "$script" ] && args=$(echo "${spec#*:}" | tr ',' ' ')
      pyk=$((pyk + 1))
      name=$(basename $script .py)_$pyk
      timeout -k 10 900 python -u $script $args > ${O}_$name.jsonl 2> ${O}_$name.err \
        || { echo PY_FAILED $script; tail -20 ${O}_$name.err; exit 1; }
      tail -c 1500 ${O}_$name.jsonl ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
