"""Every traced activity (kernels, memory copies, HIP API calls) inside a window of the last
replayed train step, from a rocprofv3 database written with --kernel-trace and optionally
--memory-copy-trace / --hip-runtime-trace — to explain idle gaps between dependent kernels that
the kernel trace alone cannot (scripts/step_sequence.py shows them as gap_us).

    python scripts/step_timeline.py OUT/run_results.db [window_start_us window_len_us]

The step is the span between the last two k_adam launches; times are printed relative to the
step's first kernel.
"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    w0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    wl = float(sys.argv[3]) if len(sys.argv) > 3 else 1500.0
    tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("# tables:", ", ".join(tables))
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    adam = [i for i, r in enumerate(rows) if "k_adam" in r[0] and "k_adam_count" not in r[0]]
    if len(adam) < 2:
        raise SystemExit("fewer than two Adam launches in the trace")
    t0 = rows[adam[-2] + 1][1]
    lo, hi = t0 + w0 * 1e3, t0 + (w0 + wl) * 1e3
    ev = []
    for t in tables:
        cols = [r[1] for r in c.execute(f"PRAGMA table_info('{t}')")]
        if "start" not in cols or "end" not in cols:
            continue
        name = next((x for x in ("name", "kernel_name", "operation", "function", "api_name") if x in cols), None)
        extra = [x for x in ("stream_id", "queue_id", "size", "dst_agent_id", "src_agent_id") if x in cols]
        sel = ", ".join(["start", "end", name or "'?'"] + extra)
        try:
            for r in c.execute(f"select {sel} from '{t}' where end >= ? and start <= ?", (lo, hi)):
                ev.append((r[0], r[1], t, str(r[2])[:70], r[3:]))
        except sqlite3.Error as e:  # noqa: PERF203 - diagnostics
            print(f"# {t}: {e}")
    if "regions" in tables:  # every graph launch of the run, relative to the step
        for st, en, nm in c.execute("select start, end, name from regions where name like 'hipGraph%' "
                                    "or name like 'hipStreamSynchronize%' order by start"):
            print(f"# api {(st - t0) / 1e3:10.1f} {(en - st) / 1e3:9.1f}  {nm}")
    ev.sort()
    for s, e, t, n, x in ev:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {t[:18]:18s} {n} {x if x else ''}")


if __name__ == "__main__":
    main()
