# Round-4 GPU step 22: PMC of the flash prefill kernel at GPT-2 B=64 T=512 after the dispatch-order change.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
export FLASH_SHAPES=0
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc22/p1 -o run -- python3 bench/probes/flash_bench.py > gpurun_out/pmc22.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc22/p2 -o run -- python3 bench/probes/flash_bench.py >> gpurun_out/pmc22.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc22 --min_grid 1 --top 3 > gpurun_out/s22_flash_pmc.md
rm -rf gpurun_out/pmc22
tail -5 gpurun_out/s22_flash_pmc.md | cut -c1-200
