"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel.

MFMA util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CUs * 4 SIMDs)
             (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy is summed over SIMDs)
wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
issue-stall= SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
LDS conflict cycles are reported per dispatch.
LDSwait%   = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES; LDSact% = SQ_LDS_IDX_ACTIVE per CU-cycle
(both only when collected: the pmcpy step of tools/gpu.sh).
"""
import collections
import csv
import sys

path = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
    per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per[name]["_dur"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

print(f"{'kernel':60s} {'n':>4s} {'us':>8s} {'MFMA%':>6s} {'wait%':>6s} {'istall%':>7s} {'LDSconf/disp':>12s} {'clkGHz':>6s}"
      f" {'LDSwait%':>8s} {'LDSact%':>7s}")
for name, c in sorted(per.items(), key=lambda kv: -sum(kv[1]["_dur"])):
    def avg(k):
        v = c.get(k)
        return sum(v) / len(v) if v else float("nan")
    n = len(c.get("GRBM_GUI_ACTIVE", [0]))
    dur = avg("_dur")
    grbm = avg("GRBM_GUI_ACTIVE")
    mfma = avg("SQ_VALU_MFMA_BUSY_CYCLES") / (grbm / 8 * 1024) * 100 if grbm else float("nan")
    wc = avg("SQ_WAVE_CYCLES")
    print(f"{name:60s} {n:4d} {dur:8.1f} {mfma:6.1f} {100*avg('SQ_WAIT_ANY')/wc:6.1f} "
          f"{100*avg('SQ_WAIT_INST_ANY')/wc:7.1f} {avg('SQ_LDS_BANK_CONFLICT'):12.0f} {grbm/8/dur/1e3:6.2f}"
          f" {100*avg('SQ_WAIT_INST_LDS')/wc:8.1f} {100*avg('SQ_LDS_IDX_ACTIVE')/(grbm/8*256) if grbm else 0:7.1f}")
