#!/bin/bash
# One GPU round-trip: gpu tests, bench, kernel-trace profile.  Run from the repo root on the box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
if [ "${PROFILE:-1}" = "1" ]; then
  R=$PWD
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-graph > $R/gpurun_out/prof_bench.log 2>&1) || exit $?
fi
if [ "${PMC:-0}" = "1" ]; then
  R=$PWD
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-graph > $R/gpurun_out/pmc_bench.log 2>&1) || exit $?
fi
