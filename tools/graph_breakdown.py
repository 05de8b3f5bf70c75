"""Per-kernel time per training step from a rocprofv3 --kernel-trace CSV of bench.py in
hipGraph mode (the timed configuration).  Steps are delimited by expand_features launches;
prints wall time, inter-kernel gaps and per-kernel microseconds averaged over the last
five complete steps.  Usage: python tools/graph_breakdown.py TRACE.csv"""
import collections
import csv
import re
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "expand_features" in r["Kernel_Name"]]
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    walls, gaps = [], []

    def name(s):
        m = re.search(r"(\w+_kernel(<[^>]*>)?|copyBuffer|FillFunctor)", s)
        return m.group(1) if m else s[:60]
    sel = range(max(0, len(starts) - 6), len(starts) - 1)
    for si in sel:
        seg = rows[starts[si]:starts[si + 1]]
        walls.append((int(rows[starts[si + 1]]["Start_Timestamp"])
                      - int(seg[0]["Start_Timestamp"])) / 1e3)
        gaps.append(sum(int(seg[i + 1]["Start_Timestamp"]) - int(seg[i]["End_Timestamp"])
                        for i in range(len(seg) - 1)) / 1e3)
        for r in seg:
            k = name(r["Kernel_Name"])
            agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
    n = len(walls)
    print(f"wall/step {sum(walls) / n:.1f} us; inter-kernel gaps {sum(gaps) / n:.1f} us/step; "
          f"{sum(cnt.values()) / n:.0f} kernels/step")
    for k, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"{k:45s} {cnt[k] / n:5.1f}/step {v / n:8.1f} us/step  avg {v / cnt[k]:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
