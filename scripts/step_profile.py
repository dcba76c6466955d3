"""Per-step kernel breakdown of the graph-replayed train step from a rocprofv3 kernel trace
of bench.py: steps are delimited by the fused Adam launch (k_adam), the last --steps of them
are averaged.  python scripts/step_profile.py gpurun_out/prof/run_kernel_trace.csv [--steps 10]"""
import argparse
import collections
import csv
import re


def category(name):
    for key, pat in (("conv fwd", r"k_conv_gemm<0|k_conv_reduce"), ("conv dgrad", r"k_conv_gemm<1"),
                     ("conv wgrad", r"k_conv_wgrad|k_reduce_splits|k_wgrad_1x1"), ("bn", r"k_bn_"),
                     ("depthwise", r"k_dw_"), ("hipBLASLt", r"Cijk_"), ("lift-splat", r"k_lss|k_target|k_tile"),
                     ("resize", r"k_resize"), ("se/pool", r"k_se_|k_avgpool|k_maxpool|k_skinny"),
                     ("adam", r"k_adam"), ("torch", r"at::native|rocclr")):
        if re.search(pat, name):
            return key
    return "other e2ep"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=35)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    ends = ends[-(a.steps + 1):]
    seg = rows[ends[0] + 1: ends[-1] + 1]
    n = len(ends) - 1
    wall = (int(rows[ends[-1]]["End_Timestamp"]) - int(rows[ends[0]]["End_Timestamp"])) / 1e6 / n
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6 / n
    print(f"{n} steps: {wall:.2f} ms/step wall, {busy:.2f} ms/step kernel time, {len(seg) / n:.0f} launches/step")
    cat = collections.defaultdict(lambda: [0.0, 0])
    ker = collections.defaultdict(lambda: [0.0, 0])
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / n
        c = category(r["Kernel_Name"])
        cat[c][0] += d
        cat[c][1] += 1
        k = r["Kernel_Name"].split("(")[0][:90]
        ker[k][0] += d
        ker[k][1] += 1
    for k, (t, m) in sorted(cat.items(), key=lambda kv: -kv[1][0]):
        print(f"{t:8.3f} ms {m / n:6.0f} launches  {k}")
    print("---")
    for k, (t, m) in sorted(ker.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t:8.3f} ms {m / n:6.0f} x {t / (m / n) * 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    main()
