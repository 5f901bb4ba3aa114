# cost of leaving 16 CUs free of stage 0 (single GPU): bench with 0 vs 16 spare CUs.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 40 > gpurun_out/sp23_0.log 2>&1 && tail -1 gpurun_out/sp23_0.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 40 --s0_spare_cus 16 > gpurun_out/sp23_16.log 2>&1 && tail -1 gpurun_out/sp23_16.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 40 > gpurun_out/sp23_0b.log 2>&1 && tail -1 gpurun_out/sp23_0b.log | cut -c1-200
