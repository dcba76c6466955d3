"""Turn a scripts/pmc_lss.sh run (gpurun_out/pmc_lss/) into profiles/lss_{fwd,bwd}_pmc.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KiB; on gfx950
FETCH_SIZE counts half the bytes of wide streaming reads, so it is doubled — MI355X_MICROARCH.md,
HBM section).  Mean kernel duration comes from the kernel-trace pass of the same run.

    python scripts/pmc_summary.py [--src gpurun_out/pmc_lss] [--batch 8] [--tag r01]"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _match(name, kernel):
    return f"::{kernel}(" in name or f"::{kernel}<" in name


def counter(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if _match(r["Kernel_Name"], kernel)]
    vals = [float(r["Counter_Value"]) for r in rows]
    return sum(vals) / len(vals) if vals else None, rows[0]["Kernel_Name"] if rows else None


def mean_ns(path, kernel):
    for r in csv.DictReader(open(path)):
        if _match(r["Name"], kernel):
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "pmc_lss"))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--tag", default="r01")
    a = ap.parse_args()
    from bench import lss_fwd_bytes, lss_bwd_bytes

    for kern, name, algo in (("k_lss_fwd", "lss_fwd", lss_fwd_bytes(a.batch)),
                             ("k_lss_bwd", "lss_bwd", lss_bwd_bytes(a.batch))):
        fetch, full = counter(os.path.join(a.src, "fetch", "run_counter_collection.csv"), kern)
        write, _ = counter(os.path.join(a.src, "write", "run_counter_collection.csv"), kern)
        ns, calls = mean_ns(os.path.join(a.src, "trace", "run_kernel_stats.csv"), kern)
        if fetch is None or write is None:
            print(f"{kern}: no counters", file=sys.stderr)
            continue
        hbm = 2 * fetch * 1024 + write * 1024
        out = {"kernel": full, "batch": a.batch, "tag": a.tag,
               "fetch_size_kib": round(fetch, 1), "write_size_kib": round(write, 1),
               "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": algo,
               "traffic_over_algorithmic": round(hbm / algo, 3),
               "rocprof_mean_ns": ns, "rocprof_calls": calls,
               "algorithmic_GBps_at_rocprof_mean": round(algo / ns, 1) if ns else None,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                         "scripts/bench_lss.py; HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB)"}
        dst = os.path.join(ROOT, "profiles", f"{name}_pmc.json")
        json.dump(out, open(dst, "w"), indent=1)
        print(dst, json.dumps(out))


if __name__ == "__main__":
    main()
