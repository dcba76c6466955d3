"""Summarise a rocprofv3 kernel_trace.csv: time per (kernel, grid) group, per step."""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: [0, 0.0])
byname = collections.defaultdict(float)
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0][:70]
    key = (short, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Grid_Size_Y"], r["Grid_Size_Z"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[key][0] += 1
    agg[key][1] += d
    byname[short] += d
tot = sum(v[1] for v in agg.values())
print(f"total {tot / steps:.1f} us/step over {len(rows)} dispatches")
print("--- by kernel name")
for k, v in sorted(byname.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v / steps:9.1f} us/step  {k}")
print("--- by (kernel, grid blocks x, y, z)")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1] / steps:9.1f} us/step n={v[0] / steps:5.1f} avg={v[1] / v[0]:8.1f}  {k}")
