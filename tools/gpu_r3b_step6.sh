# round 3 session 2, step 6: native P2P preflight fallback test, row statistics R rows per wave (tests, prefill A/B),
# GPT-2 prefill per-layer kernel sequence
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_native_comm_gpu.py tests/test_transformer_gpu.py -k "preflight or row_stats or fold or linear_norm" -x -q --timeout 200 --timeout-method thread -rs > gpurun_out/s6_tests.log 2>&1
rc=$?; tail -4 gpurun_out/s6_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s6_ab.jsonl
timeout -k 10 400 python -u bench/probes/decode_ab.py --switch rowstats_r --values 1,4 --rounds 3 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 2 --warmup 1 --prefill_iters 3 >> gpurun_out/s6_ab.jsonl 2> gpurun_out/s6_ab.err && tail -1 gpurun_out/s6_ab.jsonl || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp -o run -- python3 bench/gpt_bench.py --steps 2 --warmup 1 --prefill_iters 2 > gpurun_out/pp.log 2>&1
rc=$?
python3 tools/rocprof_seq.py gpurun_out/pp --marker flash_attn --occurrence 14 --before 3 --count 16 > gpurun_out/s6_prefill_seq.md
rm -rf gpurun_out/pp
cat gpurun_out/s6_prefill_seq.md
exit $rc
