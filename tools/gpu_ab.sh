# A/B: kernel tests + kbench + bench under two env settings ($AB_VAR = "off_value on_value")
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x > gpurun_out/ab_tests.log 2>&1 &&
timeout -k 10 300 python tools/kbench.py 2>/dev/null > gpurun_out/ab_kbench.json &&
env $AB_A timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_bench_a.log 2>&1 &&
env $AB_B timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_bench_b.log 2>&1
