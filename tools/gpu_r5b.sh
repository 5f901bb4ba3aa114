set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k "argmax_rows_step_tail or multi_step or lanes_match or gpt2_small_4stage or rowstats or large_mean or gpt2_xl_fp8_two_blocks or layernorm_q8 or fp8_split" > gpurun_out/r5b_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5b_tests.log; exit 1; }
tail -3 gpurun_out/r5b_tests.log
timeout -k 10 300 python bench/probes/decode_ab.py --switch multistep --values 1,8 --rounds 2 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5b_ab_multistep_gpt2.jsonl 2> gpurun_out/r5b_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5b_ab.err; exit 1; }
cat gpurun_out/r5b_ab_multistep_gpt2.jsonl
timeout -k 10 300 python bench/probes/decode_ab.py --switch rowstats --values 0,1 --rounds 2 --model gpt2 --stages 4 --batch 64 --prompt 512 --steps 32 --warmup 4 --prefill_iters 1 > gpurun_out/r5b_ab_rowstats_gpt2.jsonl 2>> gpurun_out/r5b_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5b_ab.err; exit 1; }
cat gpurun_out/r5b_ab_rowstats_gpt2.jsonl
timeout -k 10 300 python bench/probes/decode_ab.py --switch rowstats --values 0,1 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5b_ab_rowstats_xl.jsonl 2>> gpurun_out/r5b_ab.err || { echo AB2_FAILED; tail -20 gpurun_out/r5b_ab.err; exit 1; }
cat gpurun_out/r5b_ab_rowstats_xl.jsonl
timeout -k 10 300 python bench/probes/decode_ab.py --switch multistep --values 1,8 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 > gpurun_out/r5b_ab_multistep_xl.jsonl 2>> gpurun_out/r5b_ab.err || { echo AB3_FAILED; tail -20 gpurun_out/r5b_ab.err; exit 1; }
cat gpurun_out/r5b_ab_multistep_xl.jsonl
timeout -k 10 400 python -m distributed_neural_networks_amd.tools.fp8_fidelity --layers 2 --batch 64 --prompt 512 > gpurun_out/r5b_fp8_fidelity_2l.json 2> gpurun_out/r5b_fid.err || { echo FID_FAILED; tail -20 gpurun_out/r5b_fid.err; exit 1; }
cat gpurun_out/r5b_fp8_fidelity_2l.json
timeout -k 10 600 python bench.py > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5b_bench.err; exit 1; }
cat gpurun_out/r5b_bench.json
