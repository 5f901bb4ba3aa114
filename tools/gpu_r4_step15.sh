# Round-4 GPU step 15: PMC of the GPT-2 B=64 and GPT-2 XL fp8 B=64 decode steps on the final tree
# (one-shot GEMM, fused head), two passes each, tools/pmc_summary.py.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
for k in gpt2 xl; do
  case $k in gpt2) C=$G;; xl) C=$X;; esac
  timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_$k/p1 -o run -- python3 $C > gpurun_out/pmc15_$k.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc_$k/p2 -o run -- python3 $C >> gpurun_out/pmc15_$k.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_$k --min_grid 1 --top 12 > gpurun_out/s15_${k}_pmc.md
  rm -rf gpurun_out/pmc_$k
  tail -14 gpurun_out/s15_${k}_pmc.md | cut -c1-180
done
