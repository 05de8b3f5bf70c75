set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/profhp -o run -- python3 $R/bench.py --steps 10 --warmup 3 --secondary "" --accuracy-steps 0 > $R/gpurun_out/profhp.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/profdp -o run -- python3 $R/bench.py --steps 10 --warmup 3 --secondary "" --accuracy-steps 0 --device-pool > $R/gpurun_out/profdp.log 2>&1
