"""Diagnostic: which launch of the fused _bn1 -> swish -> SE backward differs between the bf16
storage path and the fp32 path on the same values (tests/test_bf16_store_gpu.py)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "e2e-parking-carla_amd"), os.path.join(ROOT, "tests")]
from test_bf16_store_gpu import BF, DEV, IO_DX, IO_DY, IO_X, _bfvals, _bn, _g  # noqa: E402


def cmp(tag, a, b):
    a, b = a.float(), b.float()
    d = (a - b).abs()
    print(f"{tag:40s} mismatches {int((d > 0).sum()):8d} / {a.numel():9d}  max {float(d.max()):.3e}")


def module(case):
    from e2ep_amd import nn_ops
    N, C, H, W, sq = case
    for sums in (True, False):
        nn_ops.set_se_bn_sums(sums)
        g = _g(C + sq + H)
        x = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5)
        w1 = torch.randn(sq, C, 1, 1, generator=g) / C ** 0.5
        b1 = torch.randn(sq, generator=g) * 0.1
        w2 = torch.randn(C, sq, 1, 1, generator=g) / sq ** 0.5
        b2 = torch.randn(C, generator=g) * 0.1
        for dyb in (False, True):
            dy = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
            res = []
            for dt in (torch.float32, BF):
                bn = _bn(C, _g(C))
                ts = [x.to(DEV).to(dt).requires_grad_(True)] + \
                     [t.to(DEV).requires_grad_(True) for t in (w1, b1, w2, b2)]
                y = nn_ops.bn_swish_squeeze_excite(ts[0], bn, *ts[1:])
                y.backward(dy.to(y.dtype) if dyb else dy.float())
                res.append([t.grad for t in ts] + [bn.weight.grad, bn.bias.grad])
            for i, nm in enumerate(("dx", "dw1", "db1", "dw2", "db2", "dgamma", "dbeta")):
                cmp(f"{case} sums={sums} dy_bf16={dyb} {nm}", res[1][i], res[0][i])


def bn_all(shape):
    from e2ep_amd import _lib
    lib = _lib.load()
    N, C, H, W = shape
    g = _g(C + H)
    x32 = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
    dy32 = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
    mean = (x32.mean((0, 2, 3)) + 0.01).contiguous()
    invstd = (1 / (x32.var((0, 2, 3)) + 1e-3).sqrt()).contiguous()
    gam = (1 + 0.3 * torch.randn(C, generator=g)).to(DEV)
    bet = (0.2 * torch.randn(C, generator=g)).to(DEV)
    logit = torch.randn(N, C, generator=g).to(DEV)
    dpool = torch.randn(N, C, generator=g).to(DEV)
    ws = torch.empty(max(lib.e2ep_bn_workspace(N, C, H, W), 16), dtype=torch.uint8, device=DEV)
    st = _lib.stream()
    for small in (1, 0):
        prev = _lib.call_raw("e2ep_bn_small", small)
        outs = {}
        for io, xx, dd, dt in ((0, x32, dy32, torch.float32), (7, x32.to(BF), dy32.to(BF), BF),
                               (5, x32.to(BF), dy32, BF), (2, x32, dy32.to(BF), torch.float32)):
            dx = torch.empty(N, C, H, W, device=DEV, dtype=dt)
            dg, db = torch.empty_like(gam), torch.empty_like(bet)
            _lib.call("e2ep_bn_bwd", _lib.ptr(xx), _lib.ptr(dd), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gam), _lib.ptr(bet), None, None, 1.0, _lib.ptr(logit), _lib.ptr(dpool),
                      N, C, H, W, 1, 2, _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), None, _lib.ptr(ws),
                      _lib.nbytes(ws), st, io)
            outs[io] = (dx, dg, db)
        for io in (7, 5, 2):
            cmp(f"bn_bwd {shape} small={small} io={io} dx", outs[io][0], outs[0][0].to(outs[io][0].dtype))
            cmp(f"bn_bwd {shape} small={small} io={io} dgamma", outs[io][1], outs[0][1])
        _lib.call_raw("e2ep_bn_small", prev)


def raw(case):
    """The module's launches one by one, fp32 vs bf16 storage on the same values."""
    from e2ep_amd import _lib
    N, C, H, W, sq = case
    HW = H * W
    g = _g(C + sq + H)
    x32 = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
    w1 = (torch.randn(sq, C, generator=g) / C ** 0.5).to(DEV)
    b1 = (torch.randn(sq, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(C, sq, generator=g) / sq ** 0.5).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dy32 = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
    bn = _bn(C, _g(C))
    lib = _lib.load()
    st = _lib.stream()
    outs = []
    for bf in (False, True):
        x = x32.to(BF) if bf else x32
        dy = dy32.to(BF) if bf else dy32
        rm, rv = bn.running_mean.clone(), bn.running_var.clone()
        stats = torch.empty(4, C, device=DEV)
        ws = torch.empty(max(lib.e2ep_bn_workspace(N, C, H, W), 16), dtype=torch.uint8, device=DEV)
        _lib.call("e2ep_bn_stats", _lib.ptr(x), _lib.ptr(bn.weight), _lib.ptr(bn.bias), _lib.ptr(rm),
                  _lib.ptr(rv), N, C, H, W, 1, 0.01, 1e-3, _lib.ptr(stats[0]), _lib.ptr(stats[1]),
                  _lib.ptr(stats[2]), _lib.ptr(stats[3]), _lib.ptr(ws), _lib.nbytes(ws), st,
                  IO_X if bf else 0)
        pooled, hpre, a = (torch.empty(N, C, device=DEV), torch.empty(N, sq, device=DEV),
                           torch.empty(N, C, device=DEV))
        y = torch.empty_like(x)
        _lib.call("e2ep_se_fwd", _lib.ptr(x), _lib.ptr(stats[2]), _lib.ptr(stats[3]), _lib.ptr(w1),
                  _lib.ptr(b1), _lib.ptr(w2), _lib.ptr(b2), N, C, HW, sq, _lib.ptr(pooled),
                  _lib.ptr(hpre), _lib.ptr(a), _lib.ptr(y), st, (IO_X | IO_DX) if bf else 0)
        dpooled = torch.empty(N, C, device=DEV)
        dw1, db1, dw2, db2 = (torch.empty_like(w1), torch.empty_like(b1), torch.empty_like(w2),
                              torch.empty_like(b2))
        sws = torch.empty(2 * N * C + 17 * N * sq, device=DEV)
        _lib.call("e2ep_se_bwd", _lib.ptr(x), _lib.ptr(stats[2]), _lib.ptr(stats[3]), _lib.ptr(dy),
                  _lib.ptr(w1), _lib.ptr(w2), _lib.ptr(pooled), _lib.ptr(hpre), _lib.ptr(a), N, C, HW,
                  sq, None, _lib.ptr(dpooled), _lib.ptr(dw1), _lib.ptr(db1), _lib.ptr(dw2),
                  _lib.ptr(db2), _lib.ptr(sws), st, (IO_X | IO_DY) if bf else 0)
        outs.append(dict(stats=stats, rm=rm, rv=rv, pooled=pooled, hpre=hpre, a=a, y=y.float(),
                         dpooled=dpooled, dw1=dw1, db1=db1, dw2=dw2, db2=db2))
    outs[0]["y"] = outs[0]["y"].to(BF).float()
    for k in outs[0]:
        cmp(f"raw {case} {k}", outs[1][k], outs[0][k])


def determinism(case):
    from e2ep_amd import nn_ops
    N, C, H, W, sq = case
    g = _g(C + sq + H)
    x = _bfvals(torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)
    ws_ = [torch.randn(sq, C, 1, 1, generator=g) / C ** 0.5, torch.randn(sq, generator=g) * 0.1,
           torch.randn(C, sq, 1, 1, generator=g) / sq ** 0.5, torch.randn(C, generator=g) * 0.1]
    dy = _bfvals(torch.randn(N, C, H, W, generator=g)).to(DEV)
    res = []
    for _ in range(2):
        bn = _bn(C, _g(C))
        ts = [x.clone().requires_grad_(True)] + [t.to(DEV).requires_grad_(True) for t in ws_]
        y = nn_ops.bn_swish_squeeze_excite(ts[0], bn, *ts[1:])
        y.backward(dy)
        res.append([y.detach()] + [t.grad for t in ts])
    for i, (a, b) in enumerate(zip(*res)):
        cmp(f"fp32 rerun {case} out{i}", a, b)


if __name__ == "__main__":
    for c in [(32, 672, 16, 16, 28), (8, 192, 64, 64, 8)]:
        raw(c)
        determinism(c)
    torch.cuda.synchronize()
