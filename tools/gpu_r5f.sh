# Round 5: bench with the MX prefill default + rocprofv3 kernel table of the GPT-2 XL fp8 8-stage prefill/decode.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "flash" > gpurun_out/r5f_flash_tests.log 2>&1 || { echo FLASH_TESTS_FAILED; tail -30 gpurun_out/r5f_flash_tests.log; exit 1; }
tail -2 gpurun_out/r5f_flash_tests.log
timeout -k 10 300 python bench/probes/flash_bench.py > gpurun_out/r5f_flash_bench.jsonl 2> gpurun_out/r5f_flash_bench.err || { echo FLASH_BENCH_FAILED; tail -20 gpurun_out/r5f_flash_bench.err; exit 1; }
cat gpurun_out/r5f_flash_bench.jsonl
timeout -k 10 600 python bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5f_bench.err; exit 1; }
cat gpurun_out/r5f_bench.json
timeout -k 10 300 python bench/probes/decode_ab.py --switch flash_pipe --values 0,1 --rounds 3 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 4 --warmup 1 --prefill_iters 3 > gpurun_out/r5f_ab_flash_pipe.jsonl 2> gpurun_out/r5f_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5f_ab.err; exit 1; }
cat gpurun_out/r5f_ab_flash_pipe.jsonl
X="--model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 8 --warmup 2 --prefill_iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5f -o run -- python3 bench/gpt_bench.py $X > gpurun_out/prof_r5f.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_r5f.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof_r5f > gpurun_out/r5f_xl_fp8_kernels.md
rm -rf gpurun_out/prof_r5f
head -24 gpurun_out/r5f_xl_fp8_kernels.md
