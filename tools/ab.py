"""Interleaved A/B of bench.py configurations, each run a fresh process (one at a time).

  python tools/ab.py --rounds 2 "base=" "noside=DG_SIDE_STREAM=0" "d256=|--channels,256" \
      "d256_noside=DG_SIDE_STREAM=0|--channels 256"

Each config is NAME=ENV[|BENCH ARGS] (ENV: space-separated KEY=VALUE; ARGS: space- or
comma-separated).  Prints one line per
run (name, boards/s, ms/step) as it goes and a JSON summary (best value per config) at the
end.  Every run has its own time limit; a failed run stops the A/B."""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    cfgs = []
    for c in a.configs:
        name, _, rest = c.partition("=")
        env_s, _, args_s = rest.partition("|")
        env = dict(kv.split("=", 1) for kv in env_s.split())
        cfgs.append((name, env, args_s.replace(",", " ").split()))
    res = {}
    for r in range(a.rounds):
        for name, env, args in cfgs:
            cmd = [sys.executable, os.path.join(HERE, "bench.py"), "--steps", str(a.steps),
                   "--warmup", str(a.warmup), *args]
            p = subprocess.run(cmd, env={**os.environ, **env}, capture_output=True, text=True,
                               timeout=a.timeout, cwd=HERE)
            line = [l for l in p.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
            if p.returncode != 0 or not line:
                print(f"{name}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0])
            res.setdefault(name, []).append(d["value"])
            print(f"round {r} {name:24s} {d['value']:12.1f} boards/s {d['ms_per_step']:.4f} ms",
                  flush=True)
    print(json.dumps({k: {"best": max(v), "all": v} for k, v in res.items()}))


if __name__ == "__main__":
    main()
