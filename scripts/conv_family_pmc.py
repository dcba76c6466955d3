"""HBM traffic of bench.py's headline roofline family (the conv forward + data-gradient
launches) from rocprofv3 PMC counters.

    python scripts/conv_family_pmc.py run [--precision fp32|bf16] [--passes 3]
        one eager forward + backward of the bench's train step per pass, pairs and forks off
        (as bench.py's conv_roofline times them); run it under
        rocprofv3 --pmc FETCH_SIZE (and, in a separate run, WRITE_SIZE)
        --kernel-include-regex "k_conv_(gemm|gemm2|lp|lp_reduce|reduce|direct)[<(]"
    python scripts/conv_family_pmc.py summary <fetch dir> <write dir> [--precision ...] [--passes 3]
        -> profiles/conv_family_pmc_<precision>.json: HBM bytes per step of the family
        (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md HBM section) against its algorithmic
        bytes (every launch reads its input and weights and writes its output once)."""
import argparse
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]

FAMILY = re.compile(r"k_conv_(gemm|gemm2|lp|lp_reduce|reduce|direct)[<(]")


def run(precision, passes):
    import torch
    from e2ep_amd import conv, precision as prec, synthetic
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule
    import bench
    prec.set(precision)
    torch.manual_seed(1234)
    dev = torch.device("cuda")
    mod = ParkingTrainingModule(default_cfg()).to(dev).train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    data = bench.device_batch(synthetic.synthetic_batch(8, seed=0), dev)
    step = TrainStep(mod, data, graph=False, warmup=1)
    conv.set_wgrad_overlap(False)
    conv.set_conv_pair(False)
    for _ in range(passes):
        step._fwd_bwd()
    torch.cuda.synchronize()


def algorithmic_bytes(precision):
    """Bytes per step the family must move at least: per conv launch its input, its weights
    and its output once (scripts/conv_shapes.json: the step's conv shapes and counts)."""
    shapes = json.load(open(os.path.join(ROOT, "scripts", "conv_shapes.json")))
    total = 0
    for s in shapes:
        N, Cin, H, W, Cout, R, S, P, Q = s["dims"][:9]
        gc = s.get("grad_channels") or Cin
        wts = Cout * Cin * R * S
        fwd = N * Cin * H * W + wts + N * Cout * P * Q
        dgrad = N * Cout * P * Q + Cout * gc * R * S + N * gc * H * W
        total += s["count"] * 4 * (fwd + dgrad)
    return total


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if FAMILY.search(r["Kernel_Name"]):
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


def summary(fetch_dir, write_dir, precision, passes):
    fc, wc = counters(fetch_dir), counters(write_dir)
    fetch = sum(fc.get("FETCH_SIZE", []))
    write = sum(wc.get("WRITE_SIZE", []))
    launches = len(fc.get("FETCH_SIZE", []))
    hbm = (2 * fetch + write) * 1024 / passes
    algo = algorithmic_bytes(precision)
    out = {"family": "conv forward + data gradient (bench.py roofline)", "precision": precision,
           "batch": 8, "passes": passes, "launches_per_step": launches // passes,
           "fetch_size_kib_per_step": round(fetch / passes, 1),
           "write_size_kib_per_step": round(write / passes, 1),
           "hbm_bytes_per_step": round(hbm), "algorithmic_bytes_per_step": algo,
           "traffic_over_algorithmic": round(hbm / algo, 3),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "scripts/conv_family_pmc.py run (eager fwd+bwd, pairs and forks off); HBM "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB) summed over the family's dispatches"}
    dst = os.path.join(ROOT, "profiles", f"conv_family_pmc_{precision}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("run", "summary"))
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    if a.mode == "run":
        run(a.precision, a.passes)
    else:
        summary(a.dirs[0], a.dirs[1], a.precision, a.passes)


if __name__ == "__main__":
    main()
