set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "wgrad" > gpurun_out/w3_tests.log 2>&1 &&
timeout -k 10 300 python tools/kbench.py 2>/dev/null > gpurun_out/w3_kbench.json &&
DG_WGRAD3=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/w3_bench_off.log 2>&1 &&
DG_WGRAD3=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/w3_bench_on.log 2>&1
