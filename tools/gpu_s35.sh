# Decode split A/B for GPT-2 small B=64 (default 1 split at B*Hkv >= 512) after the packed-bf16 attention.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
for s in 0 2 0 2; do
  if [ $s -eq 0 ]; then unset DNN_DECODE_SPLITS; else export DNN_DECODE_SPLITS=$s; fi
  timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/s35_$s.log 2>&1 || exit 1
  echo "splits=$s $(tail -1 gpurun_out/s35_$s.log | cut -c1-200)"
done
