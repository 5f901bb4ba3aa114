# Round 5: norm_q8 gamma/beta prefetch (tests, probe, XL prefill), GPT-2 B=64 decode gaps with medians.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "layernorm_q8 or mx or fp8_split or gpt2_xl_fp8 or norm" > gpurun_out/r5h_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5h_tests.log; exit 1; }
tail -2 gpurun_out/r5h_tests.log
timeout -k 10 200 python bench/probes/norm_q8_probe.py > gpurun_out/r5h_normq8.jsonl 2> gpurun_out/r5h_normq8.err || { echo PROBE_FAILED; tail -20 gpurun_out/r5h_normq8.err; exit 1; }
cat gpurun_out/r5h_normq8.jsonl
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 3 > gpurun_out/r5h_xl.json 2> gpurun_out/r5h_xl.err || { echo XL_FAILED; tail -20 gpurun_out/r5h_xl.err; exit 1; }
cat gpurun_out/r5h_xl.json
G="bench/gpt_bench.py --steps 16 --warmup 2 --prefill_iters 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gp_gpt2 -o run -- python3 $G > gpurun_out/gp_gpt2.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/gp_gpt2.log; exit 1; }
python3 tools/rocprof_gaps.py gpurun_out/gp_gpt2 > gpurun_out/r5h_gpt2_b64_decode_gaps.md
rm -rf gpurun_out/gp_gpt2
head -16 gpurun_out/r5h_gpt2_b64_decode_gaps.md
