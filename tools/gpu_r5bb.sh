# Round 5: what the one-shot LDS floor costs on the product decode path (interleaved A/B in one process).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench/probes/decode_ab.py --switch os_lds_floor --values 0,83968 --rounds 3 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5bb_ab_gpt2.jsonl 2> gpurun_out/r5bb.err || { echo AB1_FAILED; tail -20 gpurun_out/r5bb.err; exit 1; }
cat gpurun_out/r5bb_ab_gpt2.jsonl
timeout -k 10 400 python bench/probes/decode_ab.py --switch os_lds_floor --values 0,83968 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5bb_ab_xl.jsonl 2>> gpurun_out/r5bb.err || { echo AB2_FAILED; tail -20 gpurun_out/r5bb.err; exit 1; }
cat gpurun_out/r5bb_ab_xl.jsonl
