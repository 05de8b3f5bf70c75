# end-of-session validation: GPU suite, smoke, headline perf set, kernel trace, rocprof stats
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 &&
for cfg in "128 bf16" "128 fp8" "256 bf16" "256 fp8"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --channels $1 --dtype $2 > gpurun_out/fin_$1_$2.log 2>&1 || exit 1
done &&
timeout -k 10 200 python bench.py > gpurun_out/fin_default.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fint -o run -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/fin_t.log 2>&1
