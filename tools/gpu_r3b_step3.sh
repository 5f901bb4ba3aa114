# round 3 session 2, step 3: decode A/B with the one-pass defaults (row scores for MHA), flash prefill PMC
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s3_dec_tests.log; [ $rc -eq 0 ] || exit $rc
ab() { timeout -k 10 400 python -u bench/probes/decode_ab.py --switch decode_1p --values 0,1 "$@" >> gpurun_out/s3_ab.jsonl 2> gpurun_out/s3_ab.err && tail -1 gpurun_out/s3_ab.jsonl; }
: > gpurun_out/s3_ab.jsonl
ab --model gpt2 --stages 4 --batch 64 --prompt 512 &&
ab --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 16 --warmup 2 --prefill_iters 1 || exit 1
FLASH_SHAPES=0 timeout -k 10 120 python -u bench/probes/flash_bench.py > gpurun_out/s3_flash.log 2>&1 || exit 1
cat gpurun_out/s3_flash.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
FLASH_SHAPES=0 timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/s3_pmc1 -o run -- python3 bench/probes/flash_bench.py > gpurun_out/s3_pmc1.log 2>&1 &&
FLASH_SHAPES=0 timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/s3_pmc2 -o run -- python3 bench/probes/flash_bench.py > gpurun_out/s3_pmc2.log 2>&1
rc=$?; ls gpurun_out/s3_pmc1 gpurun_out/s3_pmc2 | head; exit $rc
