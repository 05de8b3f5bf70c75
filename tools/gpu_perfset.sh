# headline perf set: 12x128 / 12x256, bf16 / fp8
set -o pipefail
mkdir -p gpurun_out
for cfg in "128 bf16" "128 fp8" "256 bf16" "256 fp8"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --channels $1 --dtype $2 > gpurun_out/ps_$1_$2.log 2>&1 || exit 1
done
