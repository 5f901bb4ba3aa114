#!/bin/bash
# PMC passes (one rocprofv3 run per pass, no tracing domains) over a short
# program:  tools/gpu_pmc.sh <outdir> <python args...>
# Pass 1: issue/wait/MFMA busy; pass 2: LDS + L2 traffic.
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d "$out/p1" -o run -- python3 "$@" > "$out/p1.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d "$out/p2" -o run -- python3 "$@" > "$out/p2.log" 2>&1
