# Round-4 GPU step 3: fresh decode kernel tables for BASELINE configs 3, 4, 5 (rocprofv3 kernel trace) and PMC
# passes (MFMA busy, FETCH_SIZE) of the decode step and of the GPT-2 prefill GEMMs on the 256x128 / 256^2 tiles.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
for k in gpt2 xl llama; do
  case $k in gpt2) C=$G;; xl) C=$X;; llama) C=$L;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$k -o run -- python3 $C > gpurun_out/prof_$k.log 2>&1 || exit 1
  python3 tools/rocprof_summary.py gpurun_out/prof_$k > gpurun_out/s3_${k}_kernels.md
  python3 tools/rocprof_gaps.py gpurun_out/prof_$k > gpurun_out/s3_${k}_gaps.md 2>/dev/null || true
  rm -rf gpurun_out/prof_$k
  head -14 gpurun_out/s3_${k}_kernels.md | cut -c1-160
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for k in gpt2 xl; do
  case $k in gpt2) C=$G;; xl) C=$X;; esac
  timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_$k/p1 -o run -- python3 $C > gpurun_out/pmc_$k.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc_$k/p2 -o run -- python3 $C >> gpurun_out/pmc_$k.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_$k --min_grid 1 --top 10 > gpurun_out/s3_${k}_pmc.md
  rm -rf gpurun_out/pmc_$k
done
GB="bench/gemm_bench.py --tiles 255 --iters 20 --shapes 32768x768x768,32768x768x3072"
timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_gemm/p1 -o run -- python3 $GB > gpurun_out/pmc_gemm.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc_gemm/p2 -o run -- python3 $GB >> gpurun_out/pmc_gemm.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_gemm --top 6 > gpurun_out/s3_gemm255_pmc.md
rm -rf gpurun_out/pmc_gemm
GB="bench/gemm_bench.py --tiles 256 --iters 20 --shapes 32768x768x768,32768x768x3072"
timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_gemm/p1 -o run -- python3 $GB > gpurun_out/pmc_gemm.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_gemm --top 6 > gpurun_out/s3_gemm256_pmc.md
rm -rf gpurun_out/pmc_gemm
cat gpurun_out/s3_gemm255_pmc.md | head -30
timeout -k 10 200 python -u bench/probes/cifar_replay_check.py > gpurun_out/s3_cifar_replay.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench/probes/cifar_overlap_ab.py --arms 1x0,2x0,2x16 > gpurun_out/s3_cifar_overlap.jsonl 2>&1 || exit 1
grep "^{" gpurun_out/s3_cifar_*.jsonl | cut -c1-500
timeout -k 10 300 python -u bench/oneshot_sweep.py --shapes heads > gpurun_out/s3_oneshot_heads.jsonl 2>&1 || exit 1
grep "^{" gpurun_out/s3_oneshot_heads.jsonl | cut -c1-300
