#!/bin/bash
# Same-box A/B of bench.py across source trees (git worktrees with their own in-tree builds,
# e.g. .ab/<commit>): R interleaved rounds of each tree; one line per run to
# gpurun_out/ab_trees.txt.   bash tools/ab_trees.sh R "BENCH ARGS" TREE[@EXTRA ARGS]...
set -o pipefail
mkdir -p gpurun_out
R=$1; ARGS=$2; shift 2
root=$PWD
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    t=${spec%%@*}
    xa=""; case "$spec" in *@*) xa="${spec#*@}" ;; esac
    extra=""
    grep -q -- "--accuracy-steps" "$t/bench.py" && extra="--accuracy-steps 0"
    out=$(cd "$t" && timeout -k 10 300 python bench.py --steps 60 --warmup 10 $extra $ARGS $xa 2>/dev/null | grep metric) || { echo "$t failed"; exit 1; }
    echo "$spec $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k, v in d.get('secondary', {}).items()))")" | tee -a "$root/gpurun_out/ab_trees.txt"
  done
done
