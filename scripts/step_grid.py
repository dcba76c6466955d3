"""Grid-fill view of the HIP-graph-replayed train step from a rocprofv3 database: every
kernel of the timed window with its workgroup count, grouped into fill classes (a launch of
fewer workgroups than CUs leaves CUs idle while it runs, unless another stream fills them).

    python scripts/step_grid.py OUT/run_results.db [K]
Prints the columns of the kernels view (the schema varies across rocprofv3 versions), then
per fill class: launches/step, ms/step; and the kernels with the most time in small grids."""
import collections
import sqlite3
import sys


def main():
    db, K = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)")]
    print("kernels columns:", cols)
    gx = next((x for x in ("grid_x", "grid_size_x", "grid_size") if x in cols), None)
    wx = next((x for x in ("workgroup_x", "workgroup_size_x", "workgroup_size") if x in cols), None)
    gy_ = next((x for x in ("grid_y", "grid_size_y") if x in cols), None)
    gz_ = next((x for x in ("grid_z", "grid_size_z") if x in cols), None)
    wy_ = next((x for x in ("workgroup_y", "workgroup_size_y") if x in cols), None)
    wz_ = next((x for x in ("workgroup_z", "workgroup_size_z") if x in cols), None)
    if not gx or not wx:
        raise SystemExit("no grid / workgroup size columns")
    sel = ", ".join(x for x in ("name", "start", "end", gx, gy_ or "1", gz_ or "1", wx, wy_ or "1", wz_ or "1"))
    rows = c.execute(f"select {sel} from kernels order by start").fetchall()
    adam = [r for r in rows if ("k_adam(" in r[0] or r[0].startswith("e2ep::k_adam")) and "k_adam_count" not in r[0]]
    t0, t1 = adam[-K - 1][2], adam[-1][2]
    cls = collections.defaultdict(lambda: [0, 0.0])
    per = collections.defaultdict(lambda: [0, 0.0, 0])
    for name, s, e, g1, g2, g3, w1, w2, w3 in rows:
        if not (s >= t0 and e <= t1):
            continue
        wgs = (g1 // max(w1, 1)) * (g2 // max(w2, 1)) * (g3 // max(w3, 1))  # grid = threads
        if g1 < w1:  # some schemas give the grid in workgroups
            wgs = g1 * g2 * g3
        k = "<64" if wgs < 64 else "<256" if wgs < 256 else "<512" if wgs < 512 else "<1024" if wgs < 1024 else ">=1024"
        cls[k][0] += 1
        cls[k][1] += e - s
        short = name.replace("e2ep::", "").split("(")[0][:70]
        if wgs < 512:
            per[short][0] += 1
            per[short][1] += e - s
            per[short][2] = wgs
    span = (t1 - t0) / K / 1e6
    print(f"window {span:.3f} ms/step")
    for k in ("<64", "<256", "<512", "<1024", ">=1024"):
        n, t = cls[k]
        print(f"  workgroups {k:>6s}: {n / K:6.1f} launches/step {t / K / 1e6:7.3f} ms/step")
    print("kernels with < 512 workgroups, by time:")
    for name, (n, t, w) in sorted(per.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"  {t / K / 1e6:7.3f} ms {n / K:5.1f}/step  last grid {w:5d} WG  {name}")


if __name__ == "__main__":
    main()
