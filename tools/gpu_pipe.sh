# input-pipeline checks: packed loader slot copies, real-data training tests, pipeline throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_data.py tests/test_train_gpu.py -q -x -m gpu > gpurun_out/p_tests.log 2>&1 &&
timeout -k 10 200 python tools/pipeline_bench.py --threads 4 > gpurun_out/p_pipe4.log 2>&1 &&
timeout -k 10 200 python tools/pipeline_bench.py --threads 2 > gpurun_out/p_pipe2.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/p_bench.log 2>&1
