set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_win" -x -q --timeout 60 --timeout-method thread > gpurun_out/w_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -k "grouped" -x -q --timeout 60 --timeout-method thread >> gpurun_out/w_tests.log 2>&1 &&
timeout -k 10 200 python tools/kbench_win.py 128 10 > gpurun_out/kwin.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/w_b128.log 2>&1
