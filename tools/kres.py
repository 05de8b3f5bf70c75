"""Per-kernel register / spill / LDS usage of one HIP source (hipcc -Rpass-analysis=
kernel-resource-usage, gfx950).  Usage: python tools/kres.py FILE.hip [FILTER]"""
import re
import subprocess
import sys


def main(path, filt=""):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-c", path, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)",
                      line)
        if m and cur is not None:
            cur[m.group(1).split(" [")[0]] = int(m.group(2))
    if r.returncode != 0:
        print(r.stderr[-3000:])
    for c in rows:
        if filt in c["name"]:
            print(f"{c['name'][:70]:70s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} "
                  f"spill={c.get('VGPRs Spill')} lds={c.get('LDS Size')} occ={c.get('Occupancy')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
