# Decode attention with the past-context loads skipped: attention tests, then new-vs-old
# Llama-3 8B B=1 / B=32 and GPT-2 B=64 decode (old library = ab_old.so swapped in on the box copy).
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
LIB=distributed_neural_networks_amd/_dnn_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or stage or decode" > gpurun_out/k37_tests.log 2>&1; rc=$?; tail -2 gpurun_out/k37_tests.log; [ $rc -eq 0 ] || exit 1
run() {
  timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --steps 32 > gpurun_out/k37_$1_l1.log 2>&1 &&
  timeout -k 10 300 python bench/gpt_bench.py --model llama3-8b --stages 8 --batch 32 --prompt 512 --steps 16 > gpurun_out/k37_$1_l32.log 2>&1 &&
  timeout -k 10 300 python bench.py --model gpt2 > gpurun_out/k37_$1_g.log 2>&1 &&
  for f in l1 l32 g; do echo "$1 $f $(tail -1 gpurun_out/k37_$1_$f.log | cut -c1-220)"; done
}
run new && cp ab_old.so $LIB && run old && run2=1 && cp /dev/null /dev/null
