# session-4 end validation: full GPU suite, smoke, default bench x2, DP path on 1 GPU, 12x256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4_tests.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/s4_default_1.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/s4_default_2.log 2>&1 &&
timeout -k 10 200 python bench.py --force-dp > gpurun_out/s4_forcedp.log 2>&1 &&
timeout -k 10 200 python bench.py --force-dp --grad-dtype bf16 > gpurun_out/s4_forcedp_bf16.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --channels 256 > gpurun_out/s4_b256.log 2>&1
