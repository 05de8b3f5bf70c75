# full GPU tests, benches, kernel traces of 12x128 and 12x256
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/s3_b128.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/s3_b256.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --dtype fp8 > gpurun_out/s3_b128f8.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/s3t128 -o run -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/s3_t128.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/s3t256 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --channels 256 > $R/gpurun_out/s3_t256.log 2>&1
