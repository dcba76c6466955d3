"""Per-shape conv timing of the C2 train step (B=8): every conv fwd / dgrad / wgrad launch of
3 eager fwd+bwd passes bracketed by HIP events (e2ep_amd.timing, E2EP_TIMING_DETAIL=1).
Prints, per shape: launches/step, us/launch, GFLOP, TF/s, minimum HBM bytes (operands + result
once), GB/s, and which roofline bounds it (time at MFMA peak vs time at HBM peak)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT]
os.environ["E2EP_TIMING_DETAIL"] = "1"
import torch  # noqa: E402


def main():
    from e2ep_amd import conv, synthetic, timing
    conv.set_wgrad_overlap(False)  # time each weight-gradient launch alone
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule
    B = int(os.environ.get("B", "8"))
    torch.manual_seed(0)
    mod = ParkingTrainingModule(default_cfg()).cuda().train()
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    d = synthetic.synthetic_batch(B, seed=0)
    d = {k: (v if k in ("intrinsics", "extrinsics") else v.cuda()) for k, v in d.items()}
    step = TrainStep(mod, d, graph=False)
    step()
    step()
    timing.reset()
    timing.enable(True)
    n = 3
    for _ in range(n):
        step._fwd_bwd()
    timing.enable(False)
    summ, work = timing.summary(), timing.work()
    rows = []
    for k, (cnt, mean, tot) in summ.items():
        if not k.startswith("conv_"):
            continue
        kind = k.split("(")[0]
        dims = eval(k[len(kind):k.index(")") + 1])
        N, Cin, H, W, Cout, R, S, P, Q = dims[:9]
        byts = 4.0 * (N * Cin * H * W + N * Cout * P * Q + Cout * Cin * R * S)
        fl = work[k] / cnt
        us = mean * 1e3
        t_mfma = fl / 157.3e12 * 1e6
        t_hbm = byts / 8e12 * 1e6
        rows.append(dict(kind=kind, dims=list(dims), per_step=cnt / n, us=us, gflop=fl / 1e9,
                         tfs=fl / (us * 1e-6) / 1e12, mb=byts / 1e6, gbs=byts / (us * 1e-6) / 1e9,
                         bound="mfma" if t_mfma > t_hbm else "hbm",
                         frac=max(t_mfma, t_hbm) / us, ms_step=tot / n))
    rows.sort(key=lambda r: -r["ms_step"])
    tot = sum(r["ms_step"] for r in rows)
    print(f"conv total {tot:.3f} ms/step over {sum(r['per_step'] for r in rows):.0f} launches")
    print(f"{'kind':10s} {'N,Cin,H,W,Cout,R,S,P,Q,sh,sw,ph,pw,dh,dw':48s} {'n':>3s} {'us':>8s} "
          f"{'GFLOP':>7s} {'TF/s':>6s} {'MB':>7s} {'GB/s':>6s} bound  frac  ms/step")
    for r in rows[:60]:
        print(f"{r['kind']:10s} {str(r['dims']):48s} {r['per_step']:3.0f} {r['us']:8.1f} {r['gflop']:7.2f} "
              f"{r['tfs']:6.1f} {r['mb']:7.1f} {r['gbs']:6.0f} {r['bound']:5s} {r['frac']:5.2f} {r['ms_step']:7.3f}")
    out = os.environ.get("OUT")
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
