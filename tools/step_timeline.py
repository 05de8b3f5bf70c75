"""Timeline of ONE training step from a rocprofv3 --kernel-trace CSV of bench.py in hipGraph
mode: every kernel of the second-to-last complete step (steps delimited by the
feature expansion launch, or by the first layer's kernel where the expansion is fused into it) with its start offset, duration and queue, plus the busy time
of the union of all kernels (so side-stream overlap is visible).
Usage: python tools/step_timeline.py TRACE.csv [all]
  all: one step of EACH configuration in the trace (bench.py runs the headline, then the
  secondaries: the trace is cut where the step-delimiting kernel changes)"""
import csv
import re
import sys


def short(s):
    s = s.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([\w:]+(<[^>]*>)?)", s)
    return (m.group(1) if m else s)[:58]


MARKS = ("expand_features", "conv_l1_frag_kernel", "conv_stack2_kernel<1")


def main(path, every=False):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    if every:
        # configs in trace order: runs of steps sharing a step-start kernel; dp reports and
        # warmups are in the trace too, so take the 2nd-to-last step of each run
        marks = [i for i, r in enumerate(rows) if any(m in r["Kernel_Name"] for m in MARKS)]
        key = lambda i: (rows[i]["Kernel_Name"],   # noqa: E731  (+ the next launch: d = 256
                         rows[i + 1]["Kernel_Name"] if i + 1 < len(rows) else "")  # bf16 / fp8
        runs, cur = [], []
        for i in marks:
            if cur and key(i) != key(cur[-1]):
                runs.append(cur)
                cur = []
            cur.append(i)
        runs.append(cur)
        for run in runs:
            if len(run) >= 3:
                one_step(rows, run[-3], run[-2])
        return
    # a step's first launch: the feature expansion, or (fused into it) the first layer's kernel
    for mark in MARKS:
        starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
        if len(starts) >= 3:
            break
    one_step(rows, starts[-3], starts[-2])


def one_step(rows, a, b):
    seg = rows[a:b]
    t0 = int(seg[0]["Start_Timestamp"])
    wall = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
    print(f"step wall {wall:.1f} us, {len(seg)} kernels")
    print(f"{'start':>8s} {'dur':>7s} {'q':>2s}  kernel")
    iv = []
    for r in seg:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        iv.append((s, e))
        print(f"{s / 1e3:8.1f} {(e - s) / 1e3:7.1f} {r['Queue_Id']:>2s}  {short(r['Kernel_Name'])}")
    iv.sort()
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"GPU busy (union of kernels) {busy / 1e3:.1f} us = {100 * busy / 1e3 / wall:.1f}% of "
          f"the step; idle {wall - busy / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], len(sys.argv) > 2 and sys.argv[2] == "all")
