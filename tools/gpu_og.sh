# one-graph step (backward + optimizer): tests, A/B bench (12x128, 12x256), kernel trace
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_model_gpu.py tests/test_dp_gpu.py tests/test_train_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/og_tests.log 2>&1 &&
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/og_b128_$r.log 2>&1 &&
DG_ONE_GRAPH=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/og_b128_off_$r.log 2>&1 || exit 1
done &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/og_b256.log 2>&1 &&
DG_ONE_GRAPH=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/og_b256_off.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ogt -o run -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/og_t.log 2>&1
