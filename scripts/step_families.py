"""Kernel time of one replayed train step by kernel family, from a rocprofv3 kernel trace
(bench.py under rocprofv3 --kernel-trace): the window between consecutive model k_lss_fwd
launches, step index argv[2] (default 4)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_lss_fwd<" in r["Kernel_Name"]]
steps = [s for i, s in enumerate(starts) if i == 0 or s - starts[i - 1] > 5e6]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
a, b = steps[k], steps[k + 1]
fam = defaultdict(float)
busy, n = 0.0, 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not (a <= s < b):
        continue
    name = r["Kernel_Name"]
    d = (e - s) / 1e3
    busy += d
    n += 1
    key = ("hipBLASLt GEMM (transformer linears)" if "Cijk" in name
           else name.replace("void ", "").split("<")[0].split("(")[0])
    fam[key] += d
print(f"one replayed train step (step window {k}): window {(b - a) / 1e6:.2f} ms, "
      f"kernel busy {busy / 1e3:.2f} ms, {n} launches")
for key, t in sorted(fam.items(), key=lambda kv: -kv[1])[:40]:
    print(f"{t / 1e3:7.3f} ms  {key}")
