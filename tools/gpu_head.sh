set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "head" -x -q --timeout 60 --timeout-method thread > gpurun_out/h_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 60 --timeout-method thread >> gpurun_out/h_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/h_b256.log 2>&1 &&
DG_HEAD_MFMA=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/h_b256_off.log 2>&1
