"""Launch-by-launch view of one HIP-graph-replayed train step from a rocprofv3 database: the
kernels of the last step (between the last two Adam launches) in start order with their
workgroup count, duration and the idle gap since the previous launch ended — to find the
latency-bound chains (the transformer's small-row products) and the gaps between launches.

    python scripts/step_sequence.py OUT/run_results.db > step_sequence.txt
"""
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)  # drop the parameter list
    return name.replace("e2ep::", "")[:60]


def main():
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)")]
    pick = lambda *xs: next((x for x in xs if x in cols), None)  # noqa: E731
    gx, gy, gz = pick("grid_x", "grid_size_x", "grid_size"), pick("grid_y", "grid_size_y"), pick("grid_z", "grid_size_z")
    wx, wy, wz = pick("workgroup_x", "workgroup_size_x", "workgroup_size"), pick("workgroup_y", "workgroup_size_y"), pick("workgroup_z", "workgroup_size_z")
    sel = ", ".join(x or "1" for x in ("name", "start", "end", gx, gy, gz, wx, wy, wz))
    rows = c.execute(f"select {sel} from kernels order by start").fetchall()
    adam = [i for i, r in enumerate(rows) if ("k_adam(" in r[0] or "k_adam<" in r[0] or r[0].startswith("e2ep::k_adam"))
            and "k_adam_count" not in r[0]]
    if len(adam) < 2:
        raise SystemExit("fewer than two Adam launches in the trace")
    lo, hi = adam[-2] + 1, adam[-1] + 1
    prev_end = rows[adam[-2]][2]
    busy = 0
    print(f"{'#':>5} {'start_us':>9} {'dur_us':>8} {'gap_us':>7} {'WGs':>7}  kernel")
    for i in range(lo, hi):
        name, s, e, g1, g2, g3, w1, w2, w3 = rows[i]
        wgs = (g1 // max(w1, 1)) * (g2 // max(w2, 1)) * (g3 // max(w3, 1))
        if g1 < w1:
            wgs = g1 * g2 * g3
        t0 = rows[lo][1]
        print(f"{i - lo:5d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:7.1f} {wgs:7d}  {short(name)}")
        busy += e - s
        prev_end = max(prev_end, e)
    span = rows[hi - 1][2] - rows[lo][1]
    print(f"# step span {span / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, {hi - lo} launches")


if __name__ == "__main__":
    main()
