"""Summarise a rocprofv3 kernel_stats.csv (per-step microseconds)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
rows = list(csv.DictReader(open(path)))
tot = 0.0
for r in rows:
    us = float(r["TotalDurationNs"]) / 1e3 / steps
    tot += us
    print(f"{r['Name'][:80]:80s} calls/step={int(r['Calls'])/steps:6.1f} us/step={us:9.1f} avg_us={float(r['AverageNs'])/1e3:8.2f}")
print(f"TOTAL us/step = {tot:.1f}")
