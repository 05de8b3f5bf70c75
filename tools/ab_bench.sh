# A/B benchmark: alternate bench.py runs under different env settings, R rounds.
# Usage: bash tools/ab_bench.sh R "ENV_A" "ENV_B" ...   (use "-" for no extra env)
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
: > gpurun_out/ab.txt
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    e="$cfg"; [ "$e" = "-" ] && e=""
    out=$(env $e timeout -k 10 200 python bench.py --steps 60 --warmup 10 2>/dev/null | grep metric) || exit 1
    v=$(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "$cfg $v" >> gpurun_out/ab.txt
  done
done
