"""e2ep_gemm vs torch (hipBLASLt) on the transformer GEMMs of one C2 step (B = 8).

Each row: (M, N, K, layout, count per step); both sides timed with HIP events over 50
back-to-back launches on the current stream.  Prints a table and the per-step totals
(count x time), and writes JSON to --out.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "e2e-parking-carla_amd"))

import torch  # noqa: E402

# (name, M, N, K, a_kcontig, b_kcontig, launches per step); B = 8: 2048 encoder rows, 112
# decoder rows; 4 layers each
ROWS = [
    ("enc in_proj fwd", 2048, 774, 258, 1, 1, 4), ("enc in_proj dgrad", 2048, 258, 774, 1, 0, 4),
    ("enc in_proj wgrad", 774, 258, 2048, 0, 0, 4),
    ("enc out fwd", 2048, 258, 258, 1, 1, 4), ("enc out dgrad", 2048, 258, 258, 1, 0, 4),
    ("enc out wgrad", 258, 258, 2048, 0, 0, 4),
    ("enc ffn1 fwd", 2048, 2048, 258, 1, 1, 4), ("enc ffn1 dgrad", 2048, 258, 2048, 1, 0, 4),
    ("enc ffn1 wgrad", 2048, 258, 2048, 0, 0, 4),
    ("enc ffn2 fwd", 2048, 258, 2048, 1, 1, 4), ("enc ffn2 dgrad", 2048, 2048, 258, 1, 0, 4),
    ("enc ffn2 wgrad", 258, 2048, 2048, 0, 0, 4),
    ("dec self in_proj fwd", 112, 774, 258, 1, 1, 4), ("dec cross kv fwd", 2048, 516, 258, 1, 1, 4),
    ("dec cross kv dgrad", 2048, 258, 516, 1, 0, 4), ("dec cross kv wgrad", 516, 258, 2048, 0, 0, 4),
    ("dec ffn1 fwd", 112, 2048, 258, 1, 1, 4), ("dec ffn2 fwd", 112, 258, 2048, 1, 1, 4),
    ("dec ffn1 wgrad", 2048, 258, 112, 0, 0, 4), ("dec ffn2 wgrad", 258, 2048, 112, 0, 0, 4),
    ("output fwd", 112, 204, 258, 1, 1, 1),
]

# 1x1 convs of the C2 step as single-image GEMMs (N*H*W columns), --conv: (name, M, N, K,
# a_kcontig, b_kcontig, current conv kernel us from profiles/r02 conv breakdown)
CONV_ROWS = [
    ("960>160 fwd", 160, 8192, 960, 1, 0, 52.4), ("960>160 dgrad", 960, 8192, 160, 0, 0, 38.2),
    ("960>160 wgrad", 160, 960, 8192, 1, 1, 53.6),
    ("160>960 fwd", 960, 8192, 160, 1, 0, 42.1), ("160>960 dgrad", 160, 8192, 960, 0, 0, 51.9),
    ("160>960 wgrad", 960, 160, 8192, 1, 1, 53.3),
    ("672>112 fwd", 112, 8192, 672, 1, 0, 36.5), ("112>672 dgrad", 112, 8192, 672, 0, 0, 30.7),
    ("32>192 fwd", 192, 131072, 32, 1, 0, 36.7), ("192>32 wgrad", 32, 192, 131072, 1, 1, 52.2),
    ("24>144 fwd", 144, 524288, 24, 1, 0, 125.1), ("24>144 wgrad", 144, 24, 524288, 1, 1, 133.1),
    ("56>336 fwd", 336, 32768, 56, 1, 0, 34.0), ("336>56 dgrad", 336, 32768, 56, 0, 0, 30.1),
]


def torch_fn(A, ak, B, bk):
    Am = A if ak else A.t()
    Bm = B.t() if bk else B
    return lambda: torch.mm(Am, Bm)


def timed(fn, iters=50):
    """GPU time per launch (us): `iters` launches captured into one HIP graph, replayed
    between two events — no host dispatch gaps (eager back-to-back launches of these small
    GEMMs are host-bound at ~12 us)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


TILES = {1: "64x64", 2: "32x128", 3: "128x128", 4: "64x128", 5: "128x64", 6: "64x256"}


def sweep(fn):
    """Every (tile, split) plan for one shape: best six as [[us, tile, splits] ...]."""
    from e2ep_amd import _lib
    best = []
    for tile in TILES:
        for sp in (1, 2, 3, 4, 6, 8):
            _lib.call("e2ep_gemm_force", tile, sp, 0)
            best.append((timed(fn, 20), tile, sp))
    _lib.call("e2ep_gemm_force", 0, 0, 0)
    best.sort()
    print("    best:", " ".join(f"{TILES[t]}/s{sp}:{us:.1f}" for us, t, sp in best[:6]), flush=True)
    return [[round(us, 1), t, sp] for us, t, sp in best[:6]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--sweep", action="store_true", help="time every (tile, split) plan per shape")
    ap.add_argument("--conv", action="store_true", help="1x1-conv-shaped GEMMs vs the conv kernels")
    args = ap.parse_args()
    if args.conv:
        from e2ep_amd import nn_ops
        for name, M, N, K, ak, bk, conv_us in CONV_ROWS:
            A = torch.randn((M, K) if ak else (K, M), device="cuda")
            B = torch.randn((N, K) if bk else (K, N), device="cuda")
            out = torch.empty(M, N, device="cuda")
            te = timed(lambda: nn_ops.gemm(A, ak, B, bk, M, N, K, out=out))
            tt = timed(torch_fn(A, ak, B, bk))
            fl = 2.0 * M * N * K
            print(f"{name:16s} {M:6d} {N:7d} {K:7d}  e2ep {te:7.1f} us {fl / te / 1e6:6.1f} TF/s  "
                  f"torch {tt:7.1f}  conv kernel {conv_us:7.1f}", flush=True)
            if args.sweep:
                sweep(lambda: nn_ops.gemm(A, ak, B, bk, M, N, K, out=out))
        return
    from e2ep_amd import nn_ops
    rows = []
    tot_e = tot_t = 0.0
    print(f"{'gemm':24s} {'M':>5s} {'N':>5s} {'K':>5s}  {'e2ep us':>8s} {'TF/s':>6s}  {'torch us':>8s} {'TF/s':>6s}")
    for name, M, N, K, ak, bk, cnt in ROWS:
        A = torch.randn((M, K) if ak else (K, M), device="cuda")
        B = torch.randn((N, K) if bk else (K, N), device="cuda")
        out = torch.empty(M, N, device="cuda")
        te = timed(lambda: nn_ops.gemm(A, ak, B, bk, M, N, K, out=out))
        tt = timed(torch_fn(A, ak, B, bk))
        fl = 2.0 * M * N * K
        rows.append({"name": name, "M": M, "N": N, "K": K, "count": cnt, "e2ep_us": round(te, 2),
                     "torch_us": round(tt, 2), "e2ep_tflops": round(fl / te / 1e6, 1),
                     "torch_tflops": round(fl / tt / 1e6, 1)})
        tot_e += cnt * te
        tot_t += cnt * tt
        if args.sweep:
            rows[-1]["sweep"] = sweep(lambda: nn_ops.gemm(A, ak, B, bk, M, N, K, out=out))
        print(f"{name:24s} {M:5d} {N:5d} {K:5d}  {te:8.1f} {fl / te / 1e6:6.1f}  {tt:8.1f} {fl / tt / 1e6:6.1f}",
              flush=True)
    res = {"rows": rows, "per_step_ms": {"e2ep": round(tot_e / 1e3, 3), "torch": round(tot_t / 1e3, 3)}}
    print(json.dumps(res["per_step_ms"]))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
