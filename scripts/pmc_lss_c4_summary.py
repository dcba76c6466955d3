"""Turn a scripts/pmc_lss_c4.sh run into profiles/lss_c4_pmc.json (C4: B=4, 6 cams x 512^2).

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB; MI355X_MICROARCH.md HBM section), L2
hit rate = TCC_HIT / (TCC_HIT + TCC_MISS), mean duration from the kernel-trace pass.

    python scripts/pmc_lss_c4_summary.py [--src gpurun_out/pmc_lss_c4] [--tag r06]"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO = {"k_lss_fwd": 85000000.0, "k_lss_bwd": 129000000.0}  # bench.py lss_c4 bytes per launch


def _match(name, kernel):
    return f"::{kernel}(" in name or f"::{kernel}<" in name


def counters(path, kernel):
    out = {}
    for r in csv.DictReader(open(path)):
        if _match(r["Kernel_Name"], kernel):
            out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def mean_ns(path, kernel):
    for r in csv.DictReader(open(path)):
        if _match(r["Name"], kernel):
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def find(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    raise SystemExit(f"no *{suffix} under {d}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "pmc_lss_c4"))
    ap.add_argument("--tag", default="r06")
    a = ap.parse_args()
    res = {}
    for k in ("k_lss_fwd", "k_lss_bwd"):
        f = counters(find(os.path.join(a.src, "fetch"), "counter_collection.csv"), k)
        w = counters(find(os.path.join(a.src, "write"), "counter_collection.csv"), k)
        l2 = counters(find(os.path.join(a.src, "l2"), "counter_collection.csv"), k)
        ns, calls = mean_ns(find(os.path.join(a.src, "trace"), "kernel_stats.csv"), k)
        hbm = 2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024
        hit, miss = l2.get("TCC_HIT_sum"), l2.get("TCC_MISS_sum")
        res[k] = {"config": "C4: B=4, 6 cams x 512^2, 200x200 BEV (scripts/bench_lss.py --batch 4 "
                            "--cams 6 --image 512)",
                  "tag": a.tag, "fetch_size_kib": round(f["FETCH_SIZE"], 1),
                  "write_size_kib": round(w["WRITE_SIZE"], 1), "hbm_bytes_per_launch": round(hbm),
                  "algorithmic_bytes_per_launch": ALGO[k],
                  "traffic_over_algorithmic": round(hbm / ALGO[k], 3),
                  "l2_hit_rate": round(hit / (hit + miss), 3) if hit is not None else None,
                  "rocprof_mean_ns": ns, "rocprof_calls": calls,
                  "algorithmic_GBps_at_rocprof_mean": round(ALGO[k] / ns, 1) if ns else None,
                  "frac_of_8TBps": round(ALGO[k] / ns / 8000, 3) if ns else None}
    res["method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum in separate "
                     "passes (scripts/pmc_lss_c4.sh); HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB); "
                     "algorithmic bytes from scripts/bench_lss.py")
    dst = os.path.join(ROOT, "profiles", "lss_c4_pmc.json")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
