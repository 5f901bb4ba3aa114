set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log
timeout -k 10 300 python bench.py --batch 262144 --steps 10 >> gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python bench.py --steps 10 > gpurun_out/prof1.log 2>&1; echo prof rc=$?
find gpurun_out/prof1 -name "*stats*" | head
