# Round-4 GPU step 18: flash prefill with the longest query blocks dispatched first — attention GPU tests,
# flash shapes, GPT-2 prefill kernel table, bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_kv8_gpu.py tests/test_transformer_gpu.py -k "flash or qkv or attn or prefill" > gpurun_out/s18_tests.log 2>&1 || { tail -30 gpurun_out/s18_tests.log; exit 1; }
tail -2 gpurun_out/s18_tests.log
timeout -k 10 300 python bench/probes/flash_bench.py > gpurun_out/s18_flash.jsonl 2> gpurun_out/s18.err || { tail -20 gpurun_out/s18.err; exit 1; }
cat gpurun_out/s18_flash.jsonl
G="bench/gpt_bench.py --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof18 -o run -- python3 $G > gpurun_out/prof18.log 2>&1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/prof18 > gpurun_out/s18_prefill_kernels.md
rm -rf gpurun_out/prof18
grep "flash_attn" gpurun_out/s18_prefill_kernels.md | cut -c1-160
timeout -k 10 600 python bench.py > gpurun_out/s18_bench.log 2>&1 || { tail -20 gpurun_out/s18_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/s18_bench.log') if l.startswith('{')][-1])
print({k: d[k] for k in ('value','gpt2_4stage_decode_ms_per_step','gpt2_4stage_prefill_tok_s','llama3_8b_8stage_b32_decode_ms_per_step','llama3_8b_8stage_b32_prefill_tok_s','gpt2xl_fp8_8stage_b64_decode_ms_per_step','gpt2xl_fp8_8stage_b64_prefill_tok_s') if k in d})"
