# sliding-window wgrad: numerics, model equivalence, kernel sweep, bench A/B (12x128, 12x256)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_win" -x -q --timeout 60 --timeout-method thread > gpurun_out/w_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -k "grouped" -x -q --timeout 60 --timeout-method thread >> gpurun_out/w_tests.log 2>&1 &&
timeout -k 10 200 python tools/kbench_win.py 128 10 > gpurun_out/kwin.json 2>&1 &&
timeout -k 10 200 python tools/kbench_win.py 256 10 > gpurun_out/kwin256.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/w_b128.log 2>&1 &&
DG_WGRAD_WIN=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/w_b128_off.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/w_b256.log 2>&1
