# Decode-attention split sweep at Llama-3 8B B=32 (B*Hkv = 256 workgroups at one split) and GPT-2 XL fp8 B=64.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
for s in 0 1 2 4 8; do
  if [ $s -eq 0 ]; then unset DNN_DECODE_SPLITS; else export DNN_DECODE_SPLITS=$s; fi
  timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/s29_$s.log 2>&1 || exit 1
  echo "splits=$s $(tail -1 gpurun_out/s29_$s.log | cut -c1-200)"
done
