"""Per-kernel mean of every counter in a rocprofv3 --pmc counter_collection.csv (one pass of
arbitrary counters, e.g. tools/gpu.sh pmcx), with the mean dispatch time (us).

  python tools/pmc_raw.py <counter_collection.csv> [name-substring]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        name = name.split("(")[0]
        if sub not in name:
            continue
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        per[name]["_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, c in sorted(per.items(), key=lambda kv: -sum(kv[1]["_us"])):
        print(name[:90])
        print("   " + "  ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
