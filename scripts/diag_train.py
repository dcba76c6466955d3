"""Diagnostics for the captured train step: eager determinism, graph vs eager, finiteness."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from e2ep_amd import synthetic  # noqa: E402
from e2ep_amd.train import TrainStep  # noqa: E402
from tool.config import default_cfg  # noqa: E402
from trainer.pl_trainer import ParkingTrainingModule  # noqa: E402


def module(det, noise=None):
    torch.manual_seed(1234)
    m = ParkingTrainingModule(default_cfg(deterministic=det)).cuda().train()
    for p in m.parking_model.bev_encoder.layer4.parameters():
        p.requires_grad_(False)
    if noise is not None:
        m.parking_model._noise = lambda b, d, n: noise
    return m


def batch(b, seed):
    d = synthetic.synthetic_batch(b, seed=seed)
    return {k: (v if k in ("intrinsics", "extrinsics") else v.cuda()) for k, v in d.items()}


def nonfinite(m):
    bad = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
    return bad[:5], len(bad)


which = sys.argv[1] if len(sys.argv) > 1 else "all"
if which == "uaf":  # must precede every device allocation
    _so = os.path.join(ROOT, "e2e-parking-carla_amd", "e2ep_amd", "libe2ep_poison_alloc.so")
    torch.cuda.memory.change_current_allocator(
        torch.cuda.memory.CUDAPluggableAllocator(_so, "e2ep_dbg_malloc", "e2ep_dbg_free"))
if which in ("all", "det"):
    noise = synthetic.target_noise(2, seed=7).cuda()
    runs = []
    for _ in range(2):
        s = TrainStep(module(True, noise), batch(2, 7), graph=False)
        runs.append([float(s()) for _ in range(4)])
    print("eager-vs-eager", runs, flush=True)
if which in ("all", "eager"):
    s = TrainStep(module(False), batch(8, 0), graph=False)
    ls = [float(s()) for _ in range(25)]
    print("eager B=8", [round(x, 4) for x in ls], nonfinite(s.module), flush=True)
if which in ("all", "graph"):
    s = TrainStep(module(False), batch(8, 0), graph=True, warmup=5)
    ls = []
    for i in range(25):
        ls.append(float(s()))
    print("graph B=8", [round(x, 4) for x in ls], nonfinite(s.module), flush=True)


def variant(name):
    m = module(True)
    if name == "dc":
        m.parking_model.bev_model.cam_encoder.backbone.drop_connect_rate = 0.2
    elif name == "aspp":
        for mod in m.parking_model.bev_model.cam_encoder.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.5
    elif name == "tf":
        for sub in (m.parking_model.feature_fusion, m.parking_model.control_predict):
            for mod in sub.modules():
                if isinstance(mod, torch.nn.Dropout):
                    mod.p = 0.1
                if isinstance(mod, torch.nn.MultiheadAttention):
                    mod.dropout = 0.1
    return m


if which == "bisect":
    for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("noise", "dc", "aspp", "tf")):
        out = []
        for graph in (False, True):
            s = TrainStep(variant(name), batch(8, 0), graph=graph, warmup=3)
            if not graph:
                for _ in range(3):
                    s()
            out.append([round(float(s()), 3) for _ in range(4)])
        print(name, "eager", out[0], "graph", out[1], flush=True)

if which == "replay":
    m = variant(sys.argv[2] if len(sys.argv) > 2 else "noise")
    rec = []

    def _noise(b, d, n):
        t = torch.rand((b, 2), dtype=torch.float, device=d)
        rec.append(t)
        return t
    m.parking_model._noise = _noise
    ts = TrainStep(m, batch(8, 0), graph=True, warmup=3)
    W0 = ts.opt.flat.clone()
    ts.g_bwd.replay()
    torch.cuda.synchronize()
    Lg = float(ts.loss)
    Ng = rec[-1].clone()
    Gg = [p.grad.clone() for p in ts.params]
    print("graph noise", Ng.tolist(), "loss", Lg, flush=True)
    ts.g_bwd.replay()
    print("graph replay2 noise", rec[-1].tolist(), "loss", float(ts.loss), flush=True)
    ts.opt.flat.copy_(W0)
    m.parking_model._noise = lambda b, d, n: Ng.clone()
    Le = float(ts._fwd_bwd())
    Ge = [p.grad for p in ts.params]
    print("eager same noise loss", Le, flush=True)
    names = [n for n, p in m.named_parameters() if p.requires_grad]
    bad = []
    for n, a, b in zip(names, Gg, Ge):
        e = float((a - b).norm() / (b.norm() + 1e-30))
        if not e < 1e-4:
            bad.append((n, e))
    print("grad mismatches", len(bad), bad[:10], flush=True)
    for n, a, b in zip(names, Gg, Ge):
        if any(n == x[0] for x in bad):
            print(n, "graph", a.norm().item(), a.reshape(-1)[:6].tolist(), "eager", b.norm().item(),
                  b.reshape(-1)[:6].tolist(), flush=True)
    E = 258
    for n, a, b in zip(names, Gg, Ge):
        if any(n == x[0] for x in bad):
            print("slices q/k/v graph", [a[k * E:(k + 1) * E].norm().item() for k in range(3)],
                  "eager", [b[k * E:(k + 1) * E].norm().item() for k in range(3)], flush=True)
    # a second captured step in the same process, same recipe
    m2 = variant("noise")
    rec2 = []

    def _noise2(b, d, n):
        t = torch.rand((b, 2), dtype=torch.float, device=d)
        rec2.append(t)
        return t
    m2.parking_model._noise = _noise2
    ts2 = TrainStep(m2, batch(8, 0), graph=True, warmup=3)
    W2 = ts2.opt.flat.clone()
    ts2.g_bwd.replay()
    torch.cuda.synchronize()
    N2 = rec2[-1].clone()
    print("second graph: noise", N2.tolist(), "loss", float(ts2.loss), flush=True)
    ts2.opt.flat.copy_(W2)
    m2.parking_model._noise = lambda b, d, n: N2.clone()
    print("second eager same noise/weights loss", float(ts2._fwd_bwd()), flush=True)
    print("weights same as first module's W0:", torch.equal(W2, W0), flush=True)

if which == "guard":
    from e2ep_amd import debug
    noise = synthetic.target_noise(2, seed=7).cuda()
    res = {}
    for mode in ("plain", "guard"):
        if mode == "guard":
            debug.install()
        m = module(False, noise)
        torch.manual_seed(5)
        loss = m.training_step(batch(2, 7), 0)
        loss.backward()
        torch.cuda.synchronize()
        g = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        nonfin = [n for n, t in g.items() if not torch.isfinite(t).all()]
        res[mode] = (float(loss), g)
        print(mode, "loss", float(loss), "non-finite grads", len(nonfin), nonfin[:5], flush=True)
    gp, gg = res["plain"][1], res["guard"][1]
    diff = [(n, float((gg[n] - gp[n]).norm() / (gp[n].norm() + 1e-30))) for n in gp]
    diff = [d for d in diff if not d[1] < 1e-6]
    print("grad diffs plain vs guard:", len(diff), diff[:8], flush=True)

if which == "hooks":
    m = variant("noise")
    names, slots = [], {}
    sums = torch.zeros(4096, dtype=torch.float64, device="cuda")
    noise_buf = torch.zeros(8, 2, device="cuda")
    state = {"i": 0, "on": False}

    def hook(mod, inp, out):
        if not state["on"]:
            return
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for o in outs:
            if torch.is_tensor(o) and o.is_floating_point():
                i = state["i"]
                state["i"] += 1
                if len(names) <= i:
                    names.append(mod._diag_name)
                sums[i] = o.detach().abs().sum(dtype=torch.float64)

    for n, mod in m.named_modules():
        mod._diag_name = n
        if len(list(mod.children())) == 0 or n.endswith(("_blocks.0", "layer1", "layer2", "layer3")):
            mod.register_forward_hook(hook)

    def _noise(b, d, n):
        t = torch.rand((b, 2), dtype=torch.float, device=d)
        noise_buf.copy_(t)
        return t
    m.parking_model._noise = _noise
    ts = TrainStep(m, batch(8, 0), graph=False)
    for _ in range(3):
        ts()
    W0 = ts.opt.flat.clone()
    # capture now (TrainStep with graph=False: capture by hand, same as _capture)
    state["on"] = True
    state["i"] = 0
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        loss_g = ts._fwd_bwd()
    n_slots = state["i"]
    g.replay()
    torch.cuda.synchronize()
    sums_g = sums[:n_slots].clone()
    Ng = noise_buf.clone()
    Lg = float(loss_g)
    ts.opt.flat.copy_(W0)
    m.parking_model._noise = lambda b, d, n: Ng.clone()
    state["i"] = 0
    Le = float(ts._fwd_bwd())
    torch.cuda.synchronize()
    sums_e = sums[:n_slots].clone()
    print("graph loss", Lg, "eager loss", Le, "slots", n_slots, flush=True)
    rel = ((sums_g - sums_e).abs() / (sums_e.abs() + 1e-30)).tolist()
    first = [(i, names[i], r) for i, r in enumerate(rel) if r > 1e-6]
    print("first diverging:", first[:12], flush=True)

if which == "uaf":
    noise = synthetic.target_noise(2, seed=7).cuda()
    m = module(True, noise)
    for step in range(2):
        for p in m.parameters():
            p.grad = None
        loss = m.training_step(batch(2, 7), 0)
        loss.backward()
        torch.cuda.synchronize()
        bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        print("uaf step", step, "loss", float(loss), "non-finite grads", len(bad), bad[:8], flush=True)
