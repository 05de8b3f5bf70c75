set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/dp_nodp.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --force-dp > gpurun_out/dp_fp32.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --force-dp --grad-dtype bf16 > gpurun_out/dp_bf16.log 2>&1 &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dp_trun.log 2>&1
