"""Per-shape timing of the e2ep implicit-GEMM conv kernels (fwd / dgrad / wgrad separately,
back-to-back launches between HIP events) on the conv shapes of one ParkingModel train step.

    python scripts/bench_conv.py [--record] [--top 30] [--ab "6=512;6=1024"] [--precision bf16]
--record runs the model once to (re)write scripts/conv_shapes.json; --ab times every shape
under each ';'-separated e2ep_tune setting ("key=value,key=value"), interleaved in one
process, and prints the per-setting totals and per-shape times side by side."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
import torch  # noqa: E402

SHAPES = os.path.join(ROOT, "scripts", "conv_shapes.json")


def record(batch):
    from e2ep_amd import conv, synthetic
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule
    seen = {}
    orig = conv._Conv2d.apply

    def rec(x, w, b, dims, act, gc, *rest):
        key = json.dumps([list(dims), int(act), b is not None, gc])
        seen[key] = seen.get(key, 0) + 1
        return orig(x, w, b, dims, act, gc, *rest)

    conv._Conv2d.apply = rec
    mod = ParkingTrainingModule(default_cfg()).cuda().train()
    data = synthetic.synthetic_batch(batch, seed=0)
    mod.training_step(data, 0).backward()
    conv._Conv2d.apply = orig
    out = [{"dims": json.loads(k)[0], "act": json.loads(k)[1], "bias": json.loads(k)[2],
            "grad_channels": json.loads(k)[3], "count": n} for k, n in seen.items()]
    # the BEV stem's 7x7/2 conv runs inside e2ep_amd/bev_stem.py, not through conv2d
    B = batch
    out.append({"dims": [B, 65, 256, 256, 64, 7, 7, 128, 128, 2, 2, 3, 3, 1, 1], "act": 0,
                "bias": False, "grad_channels": 64, "count": 1})
    json.dump(out, open(SHAPES, "w"), indent=0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "conv_shapes.json"), "w"), indent=0)
    return out


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record", action="store_true")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--ab", default=None)
    ap.add_argument("--precision", choices=("fp32", "bf16", "fp16"), default="fp32")
    a = ap.parse_args()
    from e2ep_amd import precision
    precision.set(a.precision)
    if a.ab:
        return ab(a)
    from e2ep_amd import _lib, conv
    shapes = record(a.batch) if a.record or not os.path.exists(SHAPES) else json.load(open(SHAPES))
    rows = []
    tot = [0.0, 0.0, 0.0]
    flops_tot = 0.0
    for sh in shapes:
        d = sh["dims"]
        N, Cin, H, W, Cout, R, S, P, Q = d[:9]
        x = torch.randn(N, Cin, H, W, device="cuda")
        w = torch.randn(Cout, Cin, R, S, device="cuda")
        gy = torch.randn(N, Cout, P, Q, device="cuda")
        y = torch.empty_like(gy)
        gc = sh["grad_channels"] or Cin
        dx = torch.empty(N, gc, H, W, device="cuda")
        dw = torch.empty_like(w)
        fl = 2.0 * N * P * Q * Cout * Cin * R * S
        wt = conv.tap_major(w)
        tf = timeit(lambda: conv.conv_fwd(x, wt, None, d, sh["act"], y, w_layout=1))
        td = timeit(lambda: conv.conv_dgrad(gy, wt, d, gc, dx, w_layout=1))
        tw = timeit(lambda: conv.conv_wgrad(gy, x, d, dw))
        n = sh["count"]
        tot[0] += n * tf
        tot[1] += n * td
        tot[2] += n * tw
        flops_tot += n * 3 * fl
        rows.append((n * (tf + td + tw), n, d, tf, td, tw, fl))
    rows.sort(key=lambda r: -r[0])
    s = sum(tot)
    print(f"conv per step: fwd {tot[0]:.2f} dgrad {tot[1]:.2f} wgrad {tot[2]:.2f} = {s:.2f} ms, "
          f"{flops_tot / s / 1e9:.1f} TF/s over {len(rows)} shapes")
    print(f"{'N,Cin,H,W -> Cout,RxS /st':>34} n |   fwd  dgrad  wgrad (ms) | TF/s f / d / w")
    for tot_ms, n, d, tf, td, tw, fl in rows[:a.top]:
        desc = f"{d[0]},{d[1]},{d[2]},{d[3]}->{d[4]},{d[5]}x{d[6]}/{d[9]}"
        print(f"{desc:>34} {n:2d} | {tf:6.3f} {td:6.3f} {tw:6.3f} | {fl / tf / 1e9:5.1f} {fl / td / 1e9:5.1f} {fl / tw / 1e9:5.1f}")


def _apply(setting):
    from e2ep_amd import _lib
    lib = _lib.load()
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        if k == "v":  # conv GEMM kernel variant (e2ep_conv_gemm_variant)
            lib.e2ep_conv_gemm_variant(int(v))
        else:
            lib.e2ep_tune(int(k), int(v))


def ab(a):
    """Interleaved A/B of e2ep_tune settings per shape (fwd / dgrad / wgrad)."""
    from e2ep_amd import conv
    settings = a.ab.split(";")
    shapes = json.load(open(SHAPES))
    tot = {st: [0.0, 0.0, 0.0] for st in settings}
    rows = []
    for sh in shapes:
        d = sh["dims"]
        N, Cin, H, W, Cout, R, S, P, Q = d[:9]
        x = torch.randn(N, Cin, H, W, device="cuda")
        w = torch.randn(Cout, Cin, R, S, device="cuda")
        gy = torch.randn(N, Cout, P, Q, device="cuda")
        y = torch.empty_like(gy)
        gc = sh["grad_channels"] or Cin
        dx = torch.empty(N, gc, H, W, device="cuda")
        dw = torch.empty_like(w)
        wt = conv.tap_major(w)
        res = {}
        for rep in range(3):
            for st in settings:
                _apply(st)
                t = (timeit(lambda: conv.conv_fwd(x, wt, None, d, sh["act"], y, w_layout=1)),
                     timeit(lambda: conv.conv_dgrad(gy, wt, d, gc, dx, w_layout=1)),
                     timeit(lambda: conv.conv_wgrad(gy, x, d, dw)))
                res[st] = t if st not in res else tuple(min(u, v) for u, v in zip(res[st], t))
        n = sh["count"]
        for st in settings:
            for i in range(3):
                tot[st][i] += n * res[st][i]
        rows.append((n, d, res))
    _apply(settings[0])
    for st in settings:
        f, dg, wg = tot[st]
        print(f"[{st}] fwd {f:.3f} dgrad {dg:.3f} wgrad {wg:.3f} = {f + dg + wg:.3f} ms/step")
    for n, d, res in sorted(rows, key=lambda r: -r[0] * sum(r[2][settings[0]])):
        desc = f"{d[0]},{d[1]},{d[2]},{d[3]}->{d[4]},{d[5]}x{d[6]}/{d[9]}"
        print(f"{desc:>34} {n:2d} | " + " | ".join(
            " ".join(f"{1e3 * v:6.1f}" for v in res[st]) for st in settings))


if __name__ == "__main__":
    main()
