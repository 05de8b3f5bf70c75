# DP machinery on one GPU: RCCL world-1 tests + bench with and without the DP path, and a
# torch.distributed.run launch of the bench (driver-style) with 1 process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_dp_gpu.py -q -x > gpurun_out/dp_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/dp_bench_plain.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --force-dp > gpurun_out/dp_bench_force.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dp_bench_torchrun.log 2>&1
