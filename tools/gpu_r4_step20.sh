# Round-4 GPU step 20: kernel table of the CIFAR headline step (bench.py --no_extra) on the final tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run -- python3 bench.py --no_extra --steps 20 --warmup 5 --latency_iters 20 > gpurun_out/prof20.log 2>&1 || { tail -20 gpurun_out/prof20.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof20 > gpurun_out/s20_cifar_kernels.md
python3 tools/rocprof_gaps.py gpurun_out/prof20 > gpurun_out/s20_cifar_gaps.md 2>/dev/null || true
rm -rf gpurun_out/prof20
head -14 gpurun_out/s20_cifar_kernels.md | cut -c1-180
grep '^{' gpurun_out/prof20.log | tail -1 | cut -c1-300
