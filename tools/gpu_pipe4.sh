# trainer path with the fused (one-graph) step: train tests, real-data pipeline throughput A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_data.py tests/test_train_gpu.py tests/test_dp_gpu.py -q -x -m gpu --timeout 200 --timeout-method thread > gpurun_out/p4_tests.log 2>&1 &&
timeout -k 10 200 python tools/pipeline_bench.py --threads 4 > gpurun_out/p4_pipe.log 2>&1 &&
DG_ONE_GRAPH=0 timeout -k 10 200 python tools/pipeline_bench.py --threads 4 > gpurun_out/p4_pipe_off.log 2>&1
