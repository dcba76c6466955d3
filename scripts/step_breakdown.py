"""Per-step GPU time by kernel from a rocprofv3 kernel trace: takes the window between two
consecutive k_lss_fwd launches of the model (one train step) and sums kernel durations."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_lss_fwd<" in r["Kernel_Name"]]
# model steps: lss launches that are > 5 ms apart (the roofline loop launches back to back)
steps = [s for i, s in enumerate(starts) if i == 0 or s - starts[i - 1] > 5e6]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(steps) - 2
a, b = steps[k], steps[k + 1]
agg = defaultdict(lambda: [0.0, 0])
busy = 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if a <= s < b:
        name = r["Kernel_Name"].split("(")[0]
        agg[name][0] += (e - s) / 1e3
        agg[name][1] += 1
        busy += (e - s) / 1e3
print(f"step window {(b - a) / 1e6:.2f} ms, kernel busy {busy / 1e3:.2f} ms, launches "
      f"{sum(v[1] for v in agg.values())}")
fam = defaultdict(float)
for n, (t, c) in agg.items():
    key = n.replace("void ", "").split("<")[0]
    fam[key] += t
for n, t in sorted(fam.items(), key=lambda kv: -kv[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{t / 1e3:7.3f} ms  {n[:100]}")
