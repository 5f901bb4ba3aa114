# Decode-attention split A/B at Llama-3 8B B=1 (latency-bound: B*Hkv = 8 workgroups at one split).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
for s in 0 2 4 8; do
  if [ $s -eq 0 ]; then unset DNN_DECODE_SPLITS; else export DNN_DECODE_SPLITS=$s; fi
  timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/s26_$s.log 2>&1 || exit 1
  echo "splits=$s $(tail -1 gpurun_out/s26_$s.log | cut -c1-260)"
done
