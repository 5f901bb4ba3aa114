# Round-4 GPU step 4: the one-shot kernel with pipelined LDS steps and the wide-head exclusion —
# config re-sweep on the GPT-2 / GPT-2 XL shapes, the folded-LayerNorm path A/B (in-kernel
# statistics cost), decode A/B in the pipeline, and the Llama-3 8B decode PMC pass (FETCH_SIZE).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream_gemm_gpu.py -q --timeout 120 --timeout-method thread -x \
  > gpurun_out/s4_tests.log 2>&1 || { tail -30 gpurun_out/s4_tests.log; exit 1; }
tail -2 gpurun_out/s4_tests.log
timeout -k 10 400 python -u bench/oneshot_sweep.py --shapes gpt2,gpt2xl > gpurun_out/s4_oneshot.jsonl 2> gpurun_out/s4_oneshot.err || exit 1
grep "^{" gpurun_out/s4_oneshot.jsonl | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['N'],d['K'],d['w8'],d['dispatch_us'],d.get('best_us'),d.get('best_cfg'))"
timeout -k 10 300 python -u bench/oneshot_sweep.py --shapes gpt2,gpt2xl --epi ln,ln_gelu > gpurun_out/s4_epi.jsonl 2>> gpurun_out/s4_oneshot.err || exit 1
grep "^{" gpurun_out/s4_epi.jsonl | cut -c1-400
G="--model gpt2 --stages 4 --batch 64 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 3 $G \
  > gpurun_out/s4_ab_oneshot_gpt2.jsonl 2> gpurun_out/s4_ab.err || exit 1
tail -1 gpurun_out/s4_ab_oneshot_gpt2.jsonl | cut -c1-300
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch oneshot --values 0,1 --rounds 3 $X \
  > gpurun_out/s4_ab_oneshot_xl.jsonl 2>> gpurun_out/s4_ab.err || exit 1
tail -1 gpurun_out/s4_ab_oneshot_xl.jsonl | cut -c1-300
L="bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --warmup 2 --prefill_iters 1"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc_llama/p1 -o run -- python3 $L > gpurun_out/pmc_llama.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc_llama/p2 -o run -- python3 $L >> gpurun_out/pmc_llama.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_llama --min_grid 1 --top 10 > gpurun_out/s4_llama_pmc.md
rm -rf gpurun_out/pmc_llama
tail -12 gpurun_out/s4_llama_pmc.md | cut -c1-200
