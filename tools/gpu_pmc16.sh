# PMC counters on the flagship step (stage-0 v4, fc1 256^2 GEMM, head), 2 passes from tools/pmc_cifar.txt.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 -i tools/pmc_cifar.txt --kernel-trace --output-format csv -d gpurun_out/pmc16 -o run -- python3 bench/cifar_quick.py --batches 65536 --iters 5 > gpurun_out/pmc16.log 2>&1; echo rc=$?
ls -R gpurun_out/pmc16 | head -20
