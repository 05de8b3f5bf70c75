set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -k "stack or mask or model or grouped" -x -q --timeout 60 --timeout-method thread > gpurun_out/st_tests.log 2>&1 &&
timeout -k 10 200 python tools/kbench_stack.py > gpurun_out/kstack_s3.json 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/st_b128.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/stt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/st_t.log 2>&1
