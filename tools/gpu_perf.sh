# Quick perf loop: model/kernel GPU tests, bench (bf16), graph-mode kernel trace breakdown.
# Usage on the box: bash tools/gpu_perf.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -q -x > gpurun_out/p_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > gpurun_out/p_bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ptrace -o run -- python3 $R/bench.py --steps 10 --warmup 3 "$@" > $R/gpurun_out/p_trace.log 2>&1 &&
cd $R && python tools/graph_breakdown.py gpurun_out/ptrace/run_kernel_trace.csv > gpurun_out/p_breakdown.txt
