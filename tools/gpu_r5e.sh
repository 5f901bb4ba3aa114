set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench/probes/decode_ab.py --switch mx_prefill --values 0,1 --rounds 2 --model gpt2-xl --stages 8 --batch 64 --prompt 512 --dtype fp8 --steps 4 --warmup 1 --prefill_iters 2 > gpurun_out/r5e_ab_mx_xl.jsonl 2> gpurun_out/r5e_ab.err || { echo AB_FAILED; tail -20 gpurun_out/r5e_ab.err; exit 1; }
cat gpurun_out/r5e_ab_mx_xl.jsonl
timeout -k 10 300 python bench/probes/ring_host_probe.py --items 256 > gpurun_out/r5e_ring_host.jsonl 2> gpurun_out/r5e_ring_host.err || { echo PROBE_FAILED; tail -20 gpurun_out/r5e_ring_host.err; exit 1; }
cat gpurun_out/r5e_ring_host.jsonl
timeout -k 10 1000 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/ > gpurun_out/r5e_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5e_tests.log; exit 1; }
tail -3 gpurun_out/r5e_tests.log
