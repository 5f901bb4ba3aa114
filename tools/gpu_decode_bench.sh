#!/bin/bash
# Decode benchmarks of the transformer configs on one GPU (all stages colocated):
# GPT-2 4-stage B=64 bf16, Llama-3 8B 8-stage B=1 (bf16, fp8) and B=32, GPT-2 XL
# 8-stage fp8 B=64.  One JSON line each in gpurun_out/decode_benches.jsonl.
set -o pipefail
out=gpurun_out/decode_benches.jsonl
: > $out
run() { timeout -k 10 300 python -u bench/gpt_bench.py "$@" > gpurun_out/db.log 2>&1 && tail -1 gpurun_out/db.log >> $out; }
run --model gpt2 --stages 4 --batch 64 --prompt 512 &&
run --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 &&
run --model llama3-8b --stages 8 --batch 1 --prompt 128 &&
run --model llama3-8b --stages 8 --batch 32 --prompt 512 &&
run --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8
rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/decode_benches.jsonl"):
    d = json.loads(l)
    c = d["config"]
    print(c["model"], "B=%d" % c["micro_batch"], d["dtype"][:4], "ms/step %.4f" % d["ms_per_step"], "tok/s %.0f" % d["value"])
PY
exit $rc
