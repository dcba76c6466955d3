"""Per-step kernel time of the HIP-graph-replayed train step from a rocprofv3 database.

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 bench.py --steps K --no-cpu-baseline
    python scripts/step_kernels.py OUT/run_results.db [K] [--top N] [--csv out.csv]

The timed steps are the last K `k_adam` dispatches of the run (one optimizer update per step;
bench.py's later eager passes and lift-splat timings launch no Adam); the window runs from
the end of the (K+1)-th last `k_adam` to the end of the last one.  Prints the window's
length per step, the summed kernel time per step (their difference is GPU idle time between
kernels), and the kernels grouped by name, per step."""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("steps", type=int, nargs="?", default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--marker", default=None,
                    help="kernel name that ends each step instead of k_adam (e.g. the last kernel "
                         "of a replayed predict graph)")
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if args.marker:
        adam = [r for r in rows if args.marker in r[0]]
    else:
        adam = [r for r in rows if "k_adam(" in r[0] or r[0].startswith("e2ep::k_adam")]
        adam = [r for r in adam if "k_adam_count" not in r[0]]
    if len(adam) < args.steps + 1:
        raise SystemExit(f"only {len(adam)} marker dispatches")
    t0, t1 = adam[-args.steps - 1][2], adam[-1][2]
    K = args.steps
    per = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for name, s, e in rows:
        if s >= t0 and e <= t1:
            per[name][0] += 1
            per[name][1] += e - s
            busy += e - s
    span = (t1 - t0) / K / 1e6
    print(f"window {span:.3f} ms/step, kernel time {busy / K / 1e6:.3f} ms/step "
          f"({busy / (t1 - t0):.3f} busy), {sum(v[0] for v in per.values()) / K:.0f} launches/step")
    items = sorted(per.items(), key=lambda kv: -kv[1][1])
    print(f"{'ms/step':>8s} {'n/step':>7s} {'avg us':>8s}  kernel")
    for name, (n, t) in items[:args.top]:
        short = name.replace("e2ep::", "").split("(")[0]
        print(f"{t / K / 1e6:8.3f} {n / K:7.1f} {t / n / 1e3:8.1f}  {short[:110]}")
    if args.csv:
        with open(args.csv, "w") as f:
            f.write("kernel,launches_per_step,ms_per_step,avg_us\n")
            for name, (n, t) in items:
                f.write(f"\"{name}\",{n / K:.2f},{t / K / 1e6:.4f},{t / n / 1e3:.2f}\n")


if __name__ == "__main__":
    main()
