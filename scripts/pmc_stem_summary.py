"""Per-kernel HBM bytes of the stem A/B (scripts/pmc_stem.sh): mean FETCH_SIZE / WRITE_SIZE per
dispatch (KiB), HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section), against
the algorithmic bytes of the B = 8 stem (x 65 x 256^2 + y / gy 64 x 128^2 fp32 + 7x7x65x64 weights;
the data gradient writes 64 x 256^2 fp32).

    python scripts/pmc_stem_summary.py OUT_DIR > profiles/r06/stem_pmc.txt"""
import csv
import os
import sys

KERNELS = ["k_conv_lp<0, 0, 1, 4", "k_conv_stem_lp<", "k_conv_lp<1, 0, 1, 4", "k_conv_stem_dgrad_lp<",
           "k_wgrad_lp<1, 2, 1, 32", "k_conv_stem_wgrad_lp<"]
B = 8
X, Y, W = 4 * B * 65 * 256 * 256, 4 * B * 64 * 128 * 128, 4 * 64 * 65 * 49
ALGO = {"k_conv_lp<0, 0, 1, 4": X + Y + W, "k_conv_stem_lp<": X + Y + W,
        "k_conv_lp<1, 0, 1, 4": Y + 4 * B * 64 * 256 * 256 + W,
        "k_conv_stem_dgrad_lp<": Y + 4 * B * 64 * 256 * 256 + W,
        "k_wgrad_lp<1, 2, 1, 32": X + Y, "k_conv_stem_wgrad_lp<": X + Y}


def load(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return list(csv.DictReader(open(os.path.join(root, f))))
    raise SystemExit(f"no counter_collection.csv under {d}")


def mean(rows, k):
    v = [float(r["Counter_Value"]) for r in rows if k in r["Kernel_Name"]]
    return sum(v) / len(v) if v else None


def main():
    o = sys.argv[1]
    f, w = load(os.path.join(o, "FETCH_SIZE")), load(os.path.join(o, "WRITE_SIZE"))
    print("# kernel, FETCH_SIZE KiB, WRITE_SIZE KiB, HBM MB (2F + W), algorithmic MB, ratio")
    for k in KERNELS:
        a, b = mean(f, k), mean(w, k)
        if a is None or b is None:
            print(f"{k:28s} (no dispatch)")
            continue
        hbm = (2 * a + b) * 1024
        print(f"{k:28s} {a:12.0f} {b:12.0f} {hbm / 1e6:10.1f} {ALGO[k] / 1e6:10.1f} {hbm / ALGO[k]:6.2f}")


if __name__ == "__main__":
    main()
