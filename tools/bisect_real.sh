set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/real_data_run.py --rates 0.05 --iters 300 > gpurun_out/bis_default.log 2>&1 &&
DG_WGRAD3=0 timeout -k 10 200 python tools/real_data_run.py --rates 0.05 --iters 300 > gpurun_out/bis_nowg3.log 2>&1 &&
DG_BOARD_BM=128 timeout -k 10 200 python tools/real_data_run.py --rates 0.05 --iters 300 > gpurun_out/bis_bm128.log 2>&1
