"""ParkingModel train-step benchmark on MI355X (BASELINE.json metric).

One step = one full training step of the reference's ParkingTrainingModule
(trainer/pl_trainer.py:55-83): forward (4-cam EfficientNet encoder -> lift-splat -> BEV
encoder -> fusion -> seg/depth heads -> control decoder), the control + segmentation + depth
losses, backward, and the Adam(lr 1e-4, wd 1e-4) update (:116-121), fp32, on a synthetic
B-sample batch (4 x 256x256 cameras) that is resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W --batch B]
N>1 is launched by torch.distributed.run (one rank per GPU, RCCL over xGMI): each rank runs
B samples per step (weak scaling) and the flat gradient buffer is all-reduced (the only
exchange).  The step is captured into HIP graphs during warm-up (e2ep_amd.train.TrainStep;
--eager disables capture).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train samples/sec (4-cam frames) at B=8, 1/2/4/8 MI355X; CPU-ref baseline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s


def lss_fwd_bytes(B, N=4, C=64, D=48, hw=1024, XY=40000):
    """Algorithmic HBM bytes of one fused lift-splat forward launch:
    read featT + prob once, write the C x X x Y BEV planes once, per sample."""
    return 4 * B * (N * C * hw + N * D * hw + C * XY)


def lss_bwd_bytes(B, N=4, C=64, D=48, hw=1024, XY=40000):
    """Algorithmic HBM bytes of one lift-splat backward launch: read the BEV
    gradient, prob and features once, write grad_prob and grad_feat once, per sample."""
    return 4 * B * (C * XY + 2 * N * C * hw + 2 * N * D * hw)


def lss_fwd_kernel_ms(plan, dev, C=64, iters=50):
    """Mean duration of k_lss_fwd at the bench workload: `iters` back-to-back launches of the
    fused lift-splat forward on the model's own pillar plan, bracketed by two HIP events on
    the launch stream (torch's current stream, which _lib.stream() enqueues on).  Inputs
    are seeded synthetic softmax depths / features of the model's shapes."""
    from e2ep_amd import _lib

    B, N, D, hw, XYZ = plan.B, plan.N, plan.D, plan.h * plan.w, plan.XYZ
    g = torch.Generator(device="cpu").manual_seed(0)
    prob = torch.rand(B * N, D, hw, generator=g).softmax(1).to(dev)
    featT = torch.randn(B * N, hw, C, generator=g).to(dev)
    out = torch.empty(B, C + 1, XYZ, device=dev)

    def launch():
        _lib.call("e2ep_lss_fwd", _lib.ptr(prob), _lib.ptr(featT), _lib.ptr(plan.offsets),
                  _lib.ptr(plan.order), _lib.ptr(plan.tiles), B, N, D, hw, C, XYZ, _lib.ptr(out),
                  (C + 1) * XYZ, _lib.stream())

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        launch()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters, iters


def device_batch(data, dev):
    out = {}
    for k, v in data.items():
        # intrinsics/extrinsics stay on the host, as the dataloader / agent deliver them:
        # the 3x3 rig algebra runs on the host (bit-exact with the reference CPU path)
        out[k] = v if k in ("intrinsics", "extrinsics") else v.to(dev, non_blocking=False)
    return out


def cpu_baseline(batch, steps, threads):
    """The oracle (CPU restatement of the reference, bit-identical to it in the build
    container) running the same train step on the host cores."""
    from oracle import parking_ref as O
    from e2ep_amd import synthetic

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = O.ParkingModelRef(O.Cfg).train()
    opt = O.make_optimizer(m)
    data = synthetic.synthetic_batch(batch, seed=0)
    O.train_step(m, opt, data)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        O.train_step(m, opt, data)
    dt = time.perf_counter() - t0
    return batch * steps / dt, dt


def load_traffic(batch):
    """HBM bytes per lss_fwd launch from the committed rocprofv3 PMC summary, or None."""
    path = os.path.join(ROOT, "profiles", "lss_fwd_pmc.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        j = json.load(f)
    if int(j.get("batch", -1)) != batch:
        return None
    return float(j["hbm_bytes_per_launch"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="samples per GPU per step")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box: every rank on device 0, gloo all-reduce
    # (E2EP_BENCH_REHEARSAL=1; never used for reported numbers)
    rehearsal = os.environ.get("E2EP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from e2ep_amd import _lib, synthetic, timing
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule

    _lib.load()
    torch.manual_seed(1234)  # identical initial weights on every rank
    mod = ParkingTrainingModule(default_cfg()).to(dev).train()
    # bev_encoder.layer4 is built but never run (reference model/bev_encoder.py:21,23-36):
    # it never has a gradient, so it is kept out of the reducer and the optimizer step.
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    data = device_batch(synthetic.synthetic_batch(args.batch, seed=rank), dev)
    if world > 1:  # identical initial weights on every rank (DDP's init broadcast)
        for t in list(mod.parameters()) + list(mod.buffers()):
            dist.broadcast(t.data, 0)
    # warm-up steps (the first ones also capture the step into HIP graphs)
    step = TrainStep(mod, data, lr=mod.cfg.learning_rate, weight_decay=mod.cfg.weight_decay,
                     world=world, graph=not args.eager, warmup=max(1, args.warmup))
    if args.eager:
        for _ in range(args.warmup):
            step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-kernel HIP-event timing: a few eager steps on the same stream after the timed
    # region (graph replays cannot be bracketed per kernel from the host)
    timing.reset()
    timing.enable(True)
    for _ in range(3):
        step._fwd_bwd()
    timing.enable(False)
    kern = timing.summary()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples = world * args.batch * args.steps
    value = samples / elapsed

    mean_ms, n_fwd = lss_fwd_kernel_ms(mod.parking_model.bev_model._plan, dev)
    achieved = lss_fwd_bytes(args.batch) / (mean_ms * 1e-3) / 1e9
    traffic = load_traffic(args.batch)
    roofline = {"kernel": "e2ep::k_lss_fwd (fused depth x feature outer product + pillar pooling)",
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": lss_fwd_bytes(args.batch), "launch_ms": round(mean_ms, 5),
                "launches": n_fwd, "timing": "HIP events around back-to-back launches on the "
                                             "launch stream, model's pillar plan"}

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        v, dt = cpu_baseline(args.batch, args.cpu_steps, threads)
        base = {"value": round(v, 4), "unit": "samples/s", "cores": threads, "kind": "port",
                "sample": f"{args.cpu_steps} timed train steps (after 1 warm-up) of the oracle CPU "
                          f"restatement at B={args.batch}, 4x256^2, fp32 ({dt:.1f} s)"}

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "samples/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                "config": {"workload": "ParkingModel train step (fwd + control/seg/depth losses + bwd "
                                       "+ Adam), 4 cams x 256x256, fp32, random init",
                           "global_batch": world * args.batch, "batch_per_gpu": args.batch,
                           "parallelism": f"dp{world}"},
                "roofline": roofline, "cpu_baseline": base,
                "final_loss": round(float(loss), 4)}
        print(json.dumps(line), flush=True)
        print("kernel timing (launches, mean ms, total ms):",
              {k: (n, round(m, 4), round(t, 3)) for k, (n, m, t) in kern.items()}, file=sys.stderr)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
