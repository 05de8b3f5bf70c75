"""Overlap of comm-stream kernels with compute kernels in a rocprofv3 --kernel-trace CSV of
``bench.py --force-dp --comm proxy`` (or a real multi-GPU run): for every kernel of the
comm queue (the proxy's elementwise kernels / RCCL kernels, by name), the fraction of its
lifetime during which a compute kernel (any other queue) was also running, averaged over
the last steps.  Usage: python tools/overlap_report.py TRACE.csv [NAME_SUBSTRING]"""
import collections
import csv
import sys


def main(path, needle):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    comm = [r for r in rows if needle in r["Kernel_Name"]]
    other = [r for r in rows if needle not in r["Kernel_Name"]]
    if not comm:
        print(f"no kernel matching {needle!r}")
        return
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in other]
    tot = collections.defaultdict(lambda: [0, 0, 0])
    for r in comm[-40:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        # union of overlapping compute intervals clipped to [s, e]
        segs = sorted((max(s, a), min(e, b)) for a, b, _ in iv if a < e and b > s)
        cov, cs, ce = 0, None, None
        for a, b in segs:
            if ce is None or a > ce:
                if ce is not None:
                    cov += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        if ce is not None:
            cov += ce - cs
        who = collections.Counter(n.split("(")[0][-40:] for a, b, n in iv if a < e and b > s)
        k = (r["Queue_Id"], r["Kernel_Name"].split("(")[0][-50:])
        tot[k][0] += e - s
        tot[k][1] += cov
        tot[k][2] += 1
        tot[k].append(who.most_common(2))
    for (q, name), v in tot.items():
        print(f"queue {q} {name}: {v[2]} launches, avg {v[0] / v[2] / 1e3:.1f} us, "
              f"{100 * v[1] / max(1, v[0]):.0f}% of its time beside compute kernels; "
              f"e.g. {v[-1]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "MulFunctor")
