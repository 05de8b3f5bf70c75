# DP-path overhead on one GPU (RCCL world 1): 5-layer groups + 3 MB buckets (default) vs one
# wgrad group, vs one bucket; single-GPU path for reference
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/dpov_single.log 2>&1 &&
timeout -k 10 200 python bench.py --force-dp > gpurun_out/dpov_default.log 2>&1 &&
DG_WGRAD_GROUP=16 timeout -k 10 200 python bench.py --force-dp > gpurun_out/dpov_g16.log 2>&1 &&
timeout -k 10 200 python bench.py --force-dp --bucket-mb 100 > gpurun_out/dpov_b100.log 2>&1 &&
DG_WGRAD_GROUP=16 timeout -k 10 200 python bench.py --force-dp --bucket-mb 100 > gpurun_out/dpov_g16_b100.log 2>&1
