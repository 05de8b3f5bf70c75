# kernel + model GPU tests, bench (bf16 + fp8), graph-mode kernel trace breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x > gpurun_out/q_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/q_bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dtype fp8 > gpurun_out/q_bench_fp8.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qtrace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/q_trace.log 2>&1
