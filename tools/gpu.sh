#!/bin/bash
# One parametrised GPU-box script (run from the repo root on the box, e.g.
#   gpurun --timeout 900 -- 'bash tools/gpu.sh tests smoke bench "bench:--channels 256" prof').
# Steps run in order, each under its own time limit, and the script stops at the first
# failure (no GPU step runs after a fault, abort or timeout).  Outputs go to gpurun_out/.
#   tests            python -m pytest tests -m gpu (verbose log: gpurun_out/tests.log)
#   tests:EXPR       the same restricted with -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     python bench.py ARGS (default: --steps 50 --warmup 10); JSON appended to
#                    gpurun_out/bench.jsonl
#   prof[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS (graphs off unless ARGS
#                    says otherwise; no accuracy phase) -> gpurun_out/prof_<n>/
#   pmc[:ARGS]       rocprofv3 --kernel-trace --pmc (MFMA busy, waits, LDS conflicts, clock) of
#                    bench.py --steps 3 --warmup 1 --no-graph ARGS -> gpurun_out/pmc_<n>/ and
#                    a per-kernel summary (tools/pmc_summary.py)
#   pmcpy:SCRIPT     the pmc counters (+ LDS wait / LDS-active) over python SCRIPT (a kernel
#                    micro-benchmark) -> gpurun_out/pmcpy_<n>/ and a per-kernel summary
#   pmcx:C1,C2,..:SCRIPT  one rocprofv3 --pmc pass of the listed counters over python SCRIPT
#   list             rocprofv3 -L -> gpurun_out/counters.txt
#   py:SCRIPT ARGS   python SCRIPT ARGS (a tools/ script), stdout -> gpurun_out/py_<n>.log
#   ab:R:A|B|...     R interleaved rounds of bench.py under env settings A, B, ... ("-" = none;
#                    extra bench.py arguments from $AB_ARGS; "ENV@ARGS" adds ARGS to one arm)
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$PWD}
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  echo "== step $n: $step" | tee -a gpurun_out/steps.log
  case $kind in
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
        --timeout-method thread "${k[@]}" > gpurun_out/tests.log 2>&1
      rc=$?; tail -3 gpurun_out/tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 300 python bench.py ${arg:---steps 50 --warmup 10} \
        > gpurun_out/bench_$n.log 2>&1
      rc=$?
      grep '"metric"' gpurun_out/bench_$n.log | tee -a gpurun_out/bench.jsonl ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $R/gpurun_out/prof_$n -o run -- \
        python3 $R/bench.py --accuracy-steps 0 ${arg:---steps 10 --warmup 3} > $R/gpurun_out/prof_$n.log 2>&1)
      rc=$? ;;
    pmc)
      # 8 SQ counters (the per-pass limit) + 1 GRBM: MFMA busy, waits, LDS conflicts and the
      # LDS-wait / LDS-active columns (SQ_WAIT_INST_LDS, SQ_LDS_IDX_ACTIVE)
      C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C \
        --output-format csv -d $R/gpurun_out/pmc_$n -o run -- \
        python3 $R/bench.py --steps 3 --warmup 1 --no-graph --accuracy-steps 0 $arg > $R/gpurun_out/pmc_$n.log 2>&1)
      rc=$?
      if [ $rc = 0 ]; then
        f=$(find gpurun_out/pmc_$n -name '*counter_collection.csv' | head -1)
        python tools/pmc_summary.py "$f" > gpurun_out/pmc_$n.txt && cat gpurun_out/pmc_$n.txt
      fi ;;
    pmcpy)
      C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C \
        --output-format csv -d $R/gpurun_out/pmcpy_$n -o run -- \
        python3 $R/$arg > $R/gpurun_out/pmcpy_$n.log 2>&1)
      rc=$?
      if [ $rc = 0 ]; then
        f=$(find gpurun_out/pmcpy_$n -name '*counter_collection.csv' | head -1)
        python tools/pmc_summary.py "$f" > gpurun_out/pmcpy_$n.txt && cat gpurun_out/pmcpy_$n.txt
      fi ;;
    pmcx)
      # pmcx:COUNTERS(comma-separated):SCRIPT — one pass of the given counters over SCRIPT
      C=$(echo "${arg%%:*}" | tr ',' ' ')
      scr=${arg#*:}
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C \
        --output-format csv -d $R/gpurun_out/pmcx_$n -o run -- \
        python3 $R/$scr > $R/gpurun_out/pmcx_$n.log 2>&1)
      rc=$? ;;
    list)
      timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; rc=$? ;;
    py)
      timeout -k 10 600 python $arg > gpurun_out/py_$n.log 2>&1
      rc=$?; tail -5 gpurun_out/py_$n.log ;;
    ab)
      rounds=${arg%%:*}
      IFS='|' read -ra cfgs <<< "${arg#*:}"
      rc=0
      for r in $(seq 1 $rounds); do
        for cfg in "${cfgs[@]}"; do
          e="${cfg%%@*}"; [ "$e" = "-" ] && e=""
          xa=""; [ "$e" != "$cfg" ] || true; case "$cfg" in *@*) xa="${cfg#*@}" ;; esac
          out=$(env $e timeout -k 10 200 python bench.py --steps 60 --warmup 10 --accuracy-steps 0 ${AB_ARGS:-} $xa 2>/dev/null \
                | grep metric) || { rc=1; break 2; }
          echo "$cfg $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k, v in d.get('secondary', {}).items()))")" \
            | tee -a gpurun_out/ab.txt
        done
      done ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== step $n rc=$rc" | tee -a gpurun_out/steps.log
  [ $rc = 0 ] || exit $rc
done
