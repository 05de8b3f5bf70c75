#!/bin/bash
# rocprofv3 kernel + memory-copy traces of several bench.py variants, each in its own
# directory: bash tools/prof_cmp.sh NAME "ARGS" [NAME "ARGS"]...  (ARGS may start with
# ENV=VAL settings and a TREE: prefix to run another source tree's bench.py)
set -o pipefail
R=$PWD
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  name=$1; args=$2; shift 2
  tree=$R
  case "$args" in TREE:*) t=${args%% *}; tree=$R/${t#TREE:}; args=${args#* } ;; esac
  envs=()
  while [[ "$args" =~ ^([A-Z_0-9]+=[^ ]*)\ (.*)$ ]]; do envs+=("${BASH_REMATCH[1]}"); args=${BASH_REMATCH[2]}; done
  acc=""; grep -q -- "--accuracy-steps" "$tree/bench.py" && acc="--accuracy-steps 0"
  (cd /tmp && export TMPDIR=/tmp && env "${envs[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace \
     --output-format csv -d $R/gpurun_out/pc_$name -o run -- python3 $tree/bench.py --steps 10 --warmup 3 \
     $acc $args > $R/gpurun_out/pc_$name.log 2>&1) || exit 1
done
