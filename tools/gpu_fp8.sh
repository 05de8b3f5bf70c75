set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -q -x > gpurun_out/fp8_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/fp8_bench_bf16.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dtype fp8 > gpurun_out/fp8_bench_fp8.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/fp8_bench_bf16_256.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --channels 256 --dtype fp8 > gpurun_out/fp8_bench_fp8_256.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/f8prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-graph --dtype fp8 > $GRAFT_REPO_ROOT/gpurun_out/f8prof.log 2>&1
