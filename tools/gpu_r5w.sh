# Round 5: one-shot image sync fix (vmcnt(0) + lgkmcnt(0) + s_barrier before reading the LDS-DMA image):
# race screen, anatomy (cost vs the counted wait), decode GEMM tests, GPT-2 / GPT-2 XL decode lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench/probes/epi_race_screen.py > gpurun_out/r5w_race.jsonl 2> gpurun_out/r5w_race.err || { echo RACE_FAILED; tail -20 gpurun_out/r5w_race.err; exit 1; }
cat gpurun_out/r5w_race.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stream_gemm_gpu.py tests/test_head_gpu.py > gpurun_out/r5w_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
timeout -k 10 300 python bench/probes/oneshot_anatomy.py > gpurun_out/r5w_anat.jsonl 2> gpurun_out/r5w_anat.err || { echo ANAT_FAILED; tail -20 gpurun_out/r5w_anat.err; exit 1; }
cat gpurun_out/r5w_anat.jsonl
timeout -k 10 300 python bench/gpt_bench.py --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5w_gpt2.json 2> gpurun_out/r5w_gpt2.err || { echo GPT2_FAILED; tail -20 gpurun_out/r5w_gpt2.err; exit 1; }
cat gpurun_out/r5w_gpt2.json
timeout -k 10 300 python bench/gpt_bench.py --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5w_xl.json 2> gpurun_out/r5w_xl.err || { echo XL_FAILED; tail -20 gpurun_out/r5w_xl.err; exit 1; }
cat gpurun_out/r5w_xl.json
