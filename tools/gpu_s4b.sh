# final validation of the tree as the driver will run it: full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4b_tests.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4b_smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/s4b_default.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 --dtype fp8 > gpurun_out/s4b_256fp8.log 2>&1
