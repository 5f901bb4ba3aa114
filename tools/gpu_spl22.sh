# Llama-3 8B B=32 decode: decode-attention split count A/B (env override).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
for s in 1 2 3 6; do
DNN_DECODE_SPLITS=$s timeout -k 10 400 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 --prefill_iters 1 > gpurun_out/sp22_$s.log 2>&1 || exit 1
echo "splits=$s $(tail -1 gpurun_out/sp22_$s.log | cut -c1-200)"
done
