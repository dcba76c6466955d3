"""ParkingModel train-step benchmark on MI355X (BASELINE.json metric).

One step = one full training step of the reference's ParkingTrainingModule
(trainer/pl_trainer.py:55-83): forward (4-cam EfficientNet encoder -> lift-splat -> BEV
encoder -> fusion -> seg/depth heads -> control decoder), the control + segmentation + depth
losses, backward, and the Adam(lr 1e-4, wd 1e-4) update (:116-121), fp32, on a synthetic
B-sample batch (4 x 256x256 cameras) that is resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W --batch B] [--precision bf16] [--workload c4]
--precision bf16 is BASELINE configs[2] (C3); --workload c4 is configs[3] (6 cams x 512^2, B=4
per GPU; its own metric name, no lift-splat / step roofline entries).  The default is the
metric's configuration, configs[1] (C2).
N>1: one rank per GPU, RCCL over xGMI.  Under torch.distributed.run (WORLD_SIZE set) the ranks
are already there; from a plain command line `--gpus N` re-launches this script under
torch.distributed.run with N ranks before anything touches the GPU.  Each rank runs B samples
per step (weak scaling); the flat 78 MB gradient buffer is the only exchange.  The step is
captured into HIP graphs during warm-up (e2ep_amd.train.TrainStep): with RCCL the backward runs
as two captured segments (cut below the BEV encoder, e2ep_amd.segments) and the host issues the
stage-1 gradients' ~25 MB bucket all-reduces on a communication stream between the segment
replays, so they run during the camera-encoder backward; the stage-2 bucket follows, then the
optimizer graph (no collective is captured: e2ep_amd.train explains why).  --eager disables
capture and overlaps the bucket all-reduces with the backward from autograd hooks instead.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train samples/sec (4-cam frames) at B=8, 1/2/4/8 MI355X; CPU-ref baseline"
METRIC_C4 = "train samples/sec (6-cam 512x512 frames, C4) at B=4 per MI355X; CPU-ref baseline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 = the f32 vector rate
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 / fp16
# forward 29.94 GFLOP per 4-cam 256^2 sample (FlopCounterMode), train step
# = 3 x forward
STEP_GFLOP_PER_SAMPLE = 3 * 29.94


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


def lss_c4(dev, iters=50):
    """C4 (BASELINE configs[3]): the lift-splat pair at 6 cams x 512^2, B = 4 per GPU, 200 x 200
    BEV — the HBM-bound voxel pooling stressed at hi-res.  Mean durations of e2ep_lss_fwd /
    e2ep_lss_bwd over `iters` back-to-back launches (HIP events on the launch stream) on the
    hi-res rig's own pillar plan, and the algorithmic GB/s (lss_fwd_bytes / lss_bwd_bytes)."""
    from e2ep_amd import _lib, synthetic
    from model.bev_model import BevModel
    from tool.config import default_cfg

    cfg = default_cfg()
    cfg.final_dim = (512, 512)
    bm = BevModel(cfg).to(dev)
    B = 4
    K, E = synthetic.rig(6, 512, 512, 512)
    K = K.unsqueeze(0).expand(B, *K.shape).contiguous()
    E = E.unsqueeze(0).expand(B, *E.shape).contiguous()
    plan = bm.plan(K, E, dev)
    N, D, hw, XY, C = plan.N, plan.D, plan.h * plan.w, plan.XYZ, 64
    g = torch.Generator(device="cpu").manual_seed(0)
    prob = torch.rand(B * N, D, hw, generator=g).softmax(1).to(dev)
    featT = torch.randn(B * N, hw, C, generator=g).to(dev)
    bev = torch.empty(B, C, XY, device=dev)
    gT = torch.randn(B, XY, C, generator=g).to(dev)
    gp, gf = torch.empty_like(prob), torch.empty(B * N, C, hw, device=dev)

    def fwd():
        _lib.call("e2ep_lss_fwd", _lib.ptr(prob), _lib.ptr(featT), _lib.ptr(plan.offsets),
                  _lib.ptr(plan.order), _lib.ptr(plan.tiles), B, N, D, hw, C, XY, _lib.ptr(bev),
                  C * XY, _lib.stream())

    def bwd():
        _lib.call("e2ep_lss_bwd", _lib.ptr(gT), _lib.ptr(prob), _lib.ptr(featT),
                  _lib.ptr(plan.pillar), B, N, D, hw, C, XY, _lib.ptr(gp), _lib.ptr(gf),
                  _lib.stream())

    out = {"config": "C4: 6 cams x 512^2, B=4, 200x200 BEV, C=64, D=48", "unit": "GB/s",
           "peak": HBM_PEAK_GBS}
    for name, fn, nb in (("fwd", fwd, lss_fwd_bytes(B, N, C, D, hw, XY)),
                         ("bwd", bwd, lss_bwd_bytes(B, N, C, D, hw, XY))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        gbs = nb / (ms * 1e-3) / 1e9
        out[name] = {"launch_ms": round(ms, 5), "bytes_per_launch": nb, "achieved": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4)}
    del bm
    return out


def plan_rebuild_ms(bm, K, E, dev, iters=20):
    """Cost of NOT memoising the lift-splat plan: rig algebra + pillar index + counting sort +
    tile schedule from device-resident K / E (the agent's path, where K / E arrive on the GPU
    and the plan is rebuilt every predict).  HIP events around `iters` rebuilds."""
    Kd, Ed = K.to(dev), E.to(dev)
    for _ in range(3):
        bm.plan(Kd, Ed, dev)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        bm.plan(Kd, Ed, dev)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def device_batch(data, dev):
    out = {}
    for k, v in data.items():
        # intrinsics/extrinsics stay on the host, as the dataloader / agent deliver them:
        # the 3x3 rig algebra runs on the host (bit-exact with the reference CPU path)
        out[k] = v if k in ("intrinsics", "extrinsics") else v.to(dev, non_blocking=False)
    return out


def host_cores():
    """Threads for the CPU baseline: the CPUs this process may run on (the GPU box's CPU
    share is its affinity / OMP_NUM_THREADS, not the machine's total), and the CPU model."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, model


def cpu_baseline(batch, steps, warmup, threads, hires=False):
    """The oracle (CPU restatement of the reference, bit-identical to it in the build
    container) running the same train step on the host cores: `warmup` untimed steps, then
    the median of `steps` timed steps.  hires: the C4 rig (6 x 512^2)."""
    from oracle import parking_ref as O
    from e2ep_amd import synthetic

    class CfgC4(O.Cfg):
        final_dim = [512, 512]

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = O.ParkingModelRef(CfgC4 if hires else O.Cfg).train()
    opt = O.make_optimizer(m)
    data = synthetic.synthetic_batch(batch, seed=0, hires=hires)
    for _ in range(warmup):
        O.train_step(m, opt, data)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        O.train_step(m, opt, data)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return batch / med, med, ts


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


def load_conv_traffic(batch, lowp):
    """HBM bytes per step of the conv forward + data-gradient family from the committed
    rocprofv3 PMC summary (scripts/conv_family_pmc.py), or None."""
    path = os.path.join(ROOT, "profiles", f"conv_family_pmc_{'bf16' if lowp else 'fp32'}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        j = json.load(f)
    if int(j.get("batch", -1)) != batch:
        return None
    return j


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def relaunch(n):
    """`--gpus N` from a plain command line: start N ranks under torch.distributed.run (a
    child process; nothing here has touched the GPU) and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def train_step_rate(dev, world, rank, batch, steps, warmup, hires=False, eager=False):
    """Time `steps` replays of the captured TrainStep (fwd + 3 losses + bwd + Adam) after
    `warmup` untimed ones, bracketed by a barrier + device synchronisation on both sides, the
    elapsed time taken as the max over ranks.  Returns samples/s over all ranks, ms/step, the
    last loss and the live module / step (for the per-kernel passes)."""
    from e2ep_amd import synthetic
    from e2ep_amd.train import TrainStep
    from tool.config import default_cfg
    from trainer.pl_trainer import ParkingTrainingModule

    torch.manual_seed(1234)  # identical initial weights on every rank
    cfg = default_cfg(final_dim=[512, 512], image_crop=512) if hires else default_cfg()
    mod = ParkingTrainingModule(cfg).to(dev).train()
    # bev_encoder.layer4 is built but never run (reference model/bev_encoder.py:21,23-36):
    # it never has a gradient, so it is kept out of the reducer and the optimizer step.
    for p in mod.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    data = device_batch(synthetic.synthetic_batch(batch, seed=rank, hires=hires), dev)
    if world > 1:  # identical initial weights on every rank (DDP's init broadcast)
        for t in list(mod.parameters()) + list(mod.buffers()):
            dist.broadcast(t.data, 0)
    # warm-up steps (the first ones also capture the step into HIP graphs)
    step = TrainStep(mod, data, lr=mod.cfg.learning_rate, weight_decay=mod.cfg.weight_decay,
                     world=world, graph=not eager, warmup=max(1, warmup))
    if eager:
        for _ in range(warmup):
            step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return {"value": world * batch * steps / elapsed, "ms_per_step": elapsed / steps * 1e3,
            "loss": loss, "module": mod, "step": step}


def conv_roofline(step, lowp, n_eager=3, batch=8):
    """The headline roofline entry: the conv GEMM family (forward + data gradient), its FLOPs
    (2*N*Cout*P*Q*Cin*R*S per launch) over its summed HIP-event time in `n_eager` eager
    forward+backward passes on the launch stream after the timed region (graph replays cannot
    be bracketed per kernel from the host).  Returns (entry, per-region kernel summary)."""
    from e2ep_amd import conv, timing
    timing.reset()
    timing.enable(True)
    # serial weight gradients and no paired conv backward here: a kernel's events then time
    # that kernel alone, not its overlap with a side-stream or same-grid weight gradient (the
    # timed step runs them forked / paired)
    prev_overlap = conv.set_wgrad_overlap(False)
    prev_pair = conv.set_conv_pair(False)
    for _ in range(n_eager):
        step._fwd_bwd()
    timing.enable(False)
    conv.set_wgrad_overlap(prev_overlap)
    conv.set_conv_pair(prev_pair)
    kern = timing.summary()
    work = timing.work()
    gemm = [k for k in ("conv_fwd", "conv_dgrad") if k in kern]
    g_ms = sum(kern[k][2] for k in gemm)
    g_flop = sum(work.get(k, 0.0) for k in gemm)
    g_launch = sum(kern[k][0] for k in gemm)
    g_tfs = g_flop / (g_ms * 1e-3) / 1e12
    g_peak = BF16_MFMA_PEAK_TFS if lowp else FP32_MFMA_PEAK_TFS
    entry = {"kernel": ("e2ep::k_conv_lp (+ k_conv_gemm for M < 40 / single-step K; implicit-GEMM "
                        "conv forward + data gradient, v_mfma_f32_32x32x16_bf16, 16-bit LDS rows)"
                        if lowp else
                        "e2ep::k_conv_gemm / k_conv_gemm2 / k_conv_lp<fp32> (implicit-GEMM conv "
                        "forward + data gradient, v_mfma_f32_32x32x2_f32)") +
                       "; the step's largest kernel family",
             "bound": "mfma", "achieved": round(g_tfs, 2), "peak": g_peak,
             "unit": "TFLOP/s", "frac": round(g_tfs / g_peak, 4), "traffic": None,
             "traffic_note": "HBM bytes per step of the family (2 x FETCH_SIZE + WRITE_SIZE over its "
                             "dispatches, profiles/conv_family_pmc_<precision>.json)",
             "flop_per_step": g_flop / n_eager, "ms_per_step": round(g_ms / n_eager, 4),
             "launches_per_step": g_launch // n_eager,
             "timing": f"HIP events around every conv fwd/dgrad launch of {n_eager} eager fwd+bwd "
                       "passes on the launch stream; FLOPs = 2*N*Cout*P*Q*Cin*R*S per launch; "
                       "these passes run each data gradient as its own launch (pairs and forks "
                       "off), while the timed step runs most of them paired with their weight "
                       "gradient in one grid (k_conv_bwd_pair / k_conv_bwd_pair1x1 / "
                       "k_lp_bwd_pair), so this is a per-kernel figure, not the step's"}
    tj = load_conv_traffic(batch, lowp)
    if tj is not None:
        entry["traffic"] = tj["hbm_bytes_per_step"]
        entry["traffic_over_algorithmic"] = tj["traffic_over_algorithmic"]
    return entry, kern


def _release():
    """Return the memory of models / captured steps the caller has dropped (graph pools
    included) before the next configuration is built."""
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def secondary_c3(dev, steps, warmup):
    """BASELINE configs[2] per GPU (C3): the same B=8 train step with bf16 operands in every
    conv GEMM and transformer linear (forward, data gradient, weight gradient), fp32
    accumulation, fp32 tensors in HBM, fp32 master weights / Adam / all-reduce; samples/s and
    its conv-family roofline against the bf16 dense peak."""
    from e2ep_amd import precision
    prev = precision.set("bf16")
    try:
        r = train_step_rate(dev, 1, 0, 8, steps, warmup)
        roof, _ = conv_roofline(r["step"], True)
    finally:
        precision.set(prev)
    out = {"config": "C3 per GPU: B=8, 4 cams x 256^2, bf16 operands in the conv GEMMs and the "
                     "transformer linears (forward, "
                     "data gradient, weight gradient), fp32 accumulate / storage / optimizer",
           "value": round(r["value"], 3), "unit": "samples/s", "ms_per_step": round(r["ms_per_step"], 3),
           "steps": steps, "roofline": roof}
    del r
    _release()
    return out


def secondary_c4(dev, steps, warmup):
    """BASELINE configs[3] (C4): the full train step at 6 cams x 512^2, B=4 per GPU, fp32."""
    r = train_step_rate(dev, 1, 0, 4, steps, warmup, hires=True)
    out = {"config": "C4: train step, 6 cams x 512x512, 200x200 BEV, B=4, fp32",
           "value": round(r["value"], 3), "unit": "samples/s",
           "ms_per_step": round(r["ms_per_step"], 3), "steps": steps}
    del r
    _release()
    return out


def secondary_c5(dev, iters=200, cpu_iters=5, cpu_threads=None):
    """BASELINE configs[4] (C5): closed-loop inference — ParkingModel.predict at B=1 (encoder +
    3 autoregressive decoder passes, reference model/parking_model.py:72-78, called every
    control step at agent/parking_agent.py:385) with fp16 conv operands, captured once into a
    HIP graph; per call the inputs are copied into the captured buffers, the graph replayed
    and the device synchronised; p50 / p90 over `iters` calls.  The oracle's predict on the host
    cores beside it (p50 of `cpu_iters` calls)."""
    import numpy as np
    from e2ep_amd import graphs, precision, synthetic
    from model.parking_model import ParkingModel
    from tool.config import default_cfg

    torch.manual_seed(0)
    m = ParkingModel(default_cfg()).to(dev).eval()
    host = synthetic.synthetic_batch(1, seed=0)
    host["gt_control"] = host["gt_control"][:, :1]  # BOS: the agent's first token
    keys = ("image", "target_point", "ego_motion", "gt_control")
    static = {k: host[k].to(dev) for k in keys}
    static["intrinsics"], static["extrinsics"] = host["intrinsics"], host["extrinsics"]
    noise = synthetic.target_noise(1, seed=0).to(dev)

    def call():
        with torch.no_grad():
            return m.predict(static, noise)

    with torch.no_grad():
        tok32 = call()[0].clone()
    prev = precision.set("fp16")
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                call()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g, gout, _ = graphs.capture(call)
        ts = []
        for _ in range(iters + 10):
            t0 = time.perf_counter()
            for k in keys:
                static[k].copy_(host[k], non_blocking=True)
            g.replay()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts = np.asarray(ts[10:]) * 1e3
        same = bool(torch.equal(gout[0], tok32))
    finally:
        precision.set(prev)
    out = {"config": "C5: ParkingModel.predict, B=1, 4 cams x 256^2, fp16 conv operands, HIP graph",
           "p50_ms": round(float(np.percentile(ts, 50)), 3),
           "p90_ms": round(float(np.percentile(ts, 90)), 3), "calls": iters,
           "tokens_equal_fp32": same, "published_ait_ms_rtx5000": 74.92}
    del g, gout, m, static
    _release()
    if cpu_iters > 0:
        from oracle import parking_ref as O
        if cpu_threads:
            torch.set_num_threads(cpu_threads)
        ref = O.ParkingModelRef(O.Cfg).eval()
        cts = []
        with torch.no_grad():
            ref.predict(host)
            for _ in range(cpu_iters):
                t0 = time.perf_counter()
                ref.predict(host)
                cts.append(time.perf_counter() - t0)
        out["cpu_baseline"] = {"p50_ms": round(float(np.percentile(np.asarray(cts) * 1e3, 50)), 1),
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"p50 of {cpu_iters} oracle predict calls at B=1 fp32"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU per step (default 8; 4 for --workload c4)")
    ap.add_argument("--workload", choices=("c2", "c4"), default="c2",
                    help="c2: 4 cams x 256^2 (BASELINE configs[1], the metric's config); c4: the "
                         "hi-res rig, 6 cams x 512^2, B=4 per GPU (configs[3])")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU-baseline steps (median)")
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C3 / C4 / C5 sub-records of the default (C2, N=1) line")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32",
                    help="GEMM operands: fp32 (C2, default) or bf16 (C3: bf16 operands in the "
                         "forward, data-gradient and weight-gradient conv GEMMs and transformer "
                         "linears, fp32 accumulation, storage, optimizer and everything else)")
    args = ap.parse_args()
    hires = args.workload == "c4"
    if args.batch is None:
        args.batch = 4 if hires else 8

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # rehearsal of the N>1 path on a one-GPU box: every rank on device 0, gloo all-reduce
    # (E2EP_BENCH_REHEARSAL=1; never used for reported numbers)
    rehearsal = os.environ.get("E2EP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = None
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        backend = dist.get_backend()
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    from e2ep_amd import _lib, conv, precision, timing

    _lib.load()
    precision.set(args.precision)
    r = train_step_rate(dev, world, rank, args.batch, args.steps, args.warmup, hires,
                        eager=args.eager)
    mod, step, loss = r["module"], r["step"], r["loss"]
    grad_exchange = None
    if world > 1:
        if getattr(step, "segmented", False):
            b1, b2 = step.seg_buckets
            grad_exchange = (f"backward in 2 captured segments; {len(b1)} stage-1 buckets "
                             f"all-reduced (RCCL) during the stage-2 backward, {len(b2)} after it")
        else:
            grad_exchange = "one flat all-reduce between the backward and optimizer graphs"
    value, ms_step = r["value"], r["ms_per_step"]
    final_loss = round(float(loss), 4)
    data = step.batch

    lowp = args.precision != "fp32"
    roofline, kern = conv_roofline(step, lowp, batch=args.batch)
    step_tfs = STEP_GFLOP_PER_SAMPLE * 1e9 * args.batch / (ms_step * 1e-3) / 1e12
    step_roofline = None if hires else {"bound": "mfma", "achieved": round(step_tfs, 2), "peak": FP32_MFMA_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": round(step_tfs / FP32_MFMA_PEAK_TFS, 4),
                     "flop_per_sample": STEP_GFLOP_PER_SAMPLE * 1e9,
                     "basis": "3 x 29.94 GFLOP forward per sample (SURVEY.md §8d) x B per GPU "
                              "/ ms_per_step"}

    mean_ms, n_fwd = lss_fwd_kernel_ms(mod.parking_model.bev_model._plan, dev)
    achieved = lss_fwd_bytes(args.batch) / (mean_ms * 1e-3) / 1e9
    roofline_lss = None if hires else {"kernel": "e2ep::k_lss_fwd (fused depth x feature outer product + pillar "
                              "pooling, the north-star lift-splat kernel)",
                    "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": load_traffic(args.batch),
                    "bytes_per_launch": lss_fwd_bytes(args.batch), "launch_ms": round(mean_ms, 5),
                    "launches": n_fwd, "timing": "HIP events around back-to-back launches on the "
                                                 "launch stream, model's pillar plan",
                    "plan_rebuild_ms": round(plan_rebuild_ms(
                        mod.parking_model.bev_model, data["intrinsics"], data["extrinsics"], dev), 4),
                    "plan_note": "the train step reuses the pillar plan memoised on the host K/E "
                                 "bytes (constant rig); plan_rebuild_ms is the per-step cost if "
                                 "it were rebuilt (device K/E, the agent path)"}

    c4 = lss_c4(dev) if rank == 0 else None

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads, cpu_model = host_cores()
        # C4 CPU steps take ~4x a C2 one: a bounded sample of B=1 steps (samples/s is per sample)
        cb = 1 if hires else args.batch
        cs, cw = (3, 1) if hires else (args.cpu_steps, args.cpu_warmup)
        v, med, ts = cpu_baseline(cb, cs, cw, threads, hires)
        base = {"value": round(v, 4), "unit": "samples/s", "cores": threads, "kind": "port",
                "cpu_model": cpu_model,
                "sample": f"median of {cs} timed train steps (after {cw} warm-up) of the oracle CPU "
                          f"restatement at B={cb}, {'6x512^2' if hires else '4x256^2'}, fp32, "
                          f"{threads} threads; step times "
                          + ", ".join(f"{t:.2f}" for t in ts) + " s"}

    secondary = None
    if (rank == 0 and world == 1 and not hires and not lowp and not args.eager
            and not args.no_secondary):
        # the other BASELINE configs on this GPU, each on a fresh model (the C2 graphs freed)
        mod = step = r = data = loss = None
        _release()
        secondary = {}
        threads = host_cores()[0]
        for name, fn in (("c3", lambda: secondary_c3(dev, args.steps, args.warmup)),
                         ("c4", lambda: secondary_c4(dev, max(5, args.steps // 2), 3)),
                         ("c5", lambda: secondary_c5(dev, cpu_iters=0 if args.no_cpu_baseline
                                                     else 5, cpu_threads=threads))):
            secondary[name] = fn()
            print(f"[bench] {name}: {secondary[name]}", file=sys.stderr, flush=True)

    if rank == 0:
        line = {"metric": METRIC_C4 if hires else METRIC, "value": round(value, 3), "unit": "samples/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": "bf16" if lowp else "f32", "data": "synthetic",
                "config": {"workload": "ParkingModel train step (fwd + control/seg/depth losses + bwd "
                                       "+ Adam), " + ("6 cams x 512x512 (C4), " if hires else
                                                      "4 cams x 256x256, ") +
                                       ("bf16 operands in the conv GEMMs and transformer linears "
                                        "(forward, data gradient, weight gradient), fp32 "
                                        "accumulate and storage, fp32 optimizer and all-reduce (C3)"
                                        if lowp else "fp32") + ", random init",
                           "global_batch": world * args.batch, "batch_per_gpu": args.batch,
                           "parallelism": f"dp{world}"},
                "world": {"size": world, "backend": backend, "rehearsal": rehearsal,
                          "grad_exchange": grad_exchange},
                "roofline": roofline, "step_roofline": step_roofline, "roofline_lss": roofline_lss,
                "lss_c4": c4, "cpu_baseline": base, "final_loss": final_loss,
                "secondary": secondary}
        print(json.dumps(line), flush=True)
        print("kernel timing (launches, mean ms, total ms):",
              {k: (n, round(m, 4), round(t, 3)) for k, (n, m, t) in kern.items()}, file=sys.stderr)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
