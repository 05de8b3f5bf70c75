set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py tests/test_dp_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/fh_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "head" -x -q --timeout 60 --timeout-method thread >> gpurun_out/fh_tests.log 2>&1 &&
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/fh_b128_$r.log 2>&1 &&
DG_FUSE_HEAD=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/fh_b128_off_$r.log 2>&1 || exit 1
done &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fht -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/fh_t.log 2>&1
