"""Lift-splat on MI355X: geometry/pillar plan + fused outer-product pooling (autograd op).

Python surface over the C ABI (include/e2ep.h).  Replaces, in the reference:
  model/bev_model.py:45-57   BevModel.get_geometry
  model/bev_model.py:59-71   the depth x feature outer product in encoder_forward
  model/bev_model.py:74-107  BevModel.proj_bev_feature
  tool/geometry.py:285-317   VoxelsSumming
"""
import os
from dataclasses import dataclass

import torch

from . import _lib, timing


def _require_device(*ts):
    for t in ts:
        if not t.is_cuda:
            raise _lib.E2EPError("e2ep lift-splat runs on a HIP device only; got a CPU tensor")


def plan_cache_enabled():
    return os.environ.get("E2EP_PLAN_CACHE", "1") != "0"


def rig_transforms(intrinsics, extrinsics, device):
    """combine = R(E^-1) K^-1 and trans = t(E^-1) (model/bev_model.py:46-53) on the device
    (e2ep_rig_transforms: fp64 Gauss-Jordan, one fp32 rounding; deterministic on any host).
    Returns device tensors (B,N,3,3), (B,N,3)."""
    K = intrinsics.detach().to(device=device, dtype=torch.float32).contiguous()
    E = extrinsics.detach().to(device=device, dtype=torch.float32).contiguous()
    B, N = K.shape[:2]
    combine = torch.empty(B, N, 3, 3, dtype=torch.float32, device=device)
    trans = torch.empty(B, N, 3, dtype=torch.float32, device=device)
    _lib.call("e2ep_rig_transforms", _lib.ptr(K), _lib.ptr(E), B * N, _lib.ptr(combine),
              _lib.ptr(trans), _lib.stream())
    return combine, trans


def rig_transforms_host(intrinsics, extrinsics):
    """The reference's own fp32 CPU algebra, op for op (model/bev_model.py:46-53:
    torch.inverse(E), R = inv[..., :3, :3], t = inv[..., :3, 3], R.matmul(torch.inverse(K))) on
    the dense (B,N,·,·) batch the data loader collates.  Used for host-resident rigs (the
    dataloader / agent path, memoised), so the pillar index is the reference's bit for bit on
    the same host: its last ulp comes from the host CPU's LAPACK kernels, which the fp64 device
    algebra (rig_transforms) cannot reproduce.  Returns CPU tensors."""
    K = intrinsics.detach().float().cpu().contiguous()
    E = extrinsics.detach().float().cpu().contiguous()
    inv_e = torch.inverse(E)
    combine = inv_e[..., :3, :3].matmul(torch.inverse(K))
    return combine.contiguous(), inv_e[..., :3, 3].contiguous()


@dataclass
class LssPlan:
    """Per-batch pillar plan: integer pillar of every point and the points sorted by pillar."""
    pillar: torch.Tensor   # int32 [B*N*D*h*w], -1 = masked
    offsets: torch.Tensor  # int32 [B*(XYZ+1)]
    order: torch.Tensor    # int32 [B*N*D*h*w] packed point codes
    tiles: torch.Tensor    # int32 [B*ntiles] forward tile schedule (heaviest first)
    B: int
    N: int
    D: int
    h: int
    w: int
    X: int
    Y: int
    Z: int

    @property
    def XYZ(self):
        return self.X * self.Y * self.Z


def build_plan(frustum, combine, trans, lo, res, dims, device):
    """Geometry + pillar index + counting sort on the GPU (e2ep_geom_index, e2ep_lss_plan).

    frustum: (D,h,w,3) tensor (any device); combine (B,N,3,3), trans (B,N,3) (any device);
    lo, res: 3 floats (host); dims: (X, Y, Z) ints."""
    D, h, w, _ = frustum.shape
    B, N = combine.shape[:2]
    X, Y, Z = (int(v) for v in dims)
    fr = frustum.detach().to(device=device, dtype=torch.float32).contiguous()
    cb = combine.to(device=device, dtype=torch.float32, non_blocking=True).contiguous()
    tr = trans.to(device=device, dtype=torch.float32, non_blocking=True).contiguous()
    P = N * D * h * w
    XYZ = X * Y * Z
    pillar = torch.empty(B * P, dtype=torch.int32, device=device)
    s = _lib.stream()
    _lib.call("e2ep_geom_index", _lib.ptr(fr), _lib.ptr(cb), _lib.ptr(tr), _lib.host3(lo),
              _lib.host3(res), X, Y, Z, B, N, D, h, w, _lib.ptr(pillar), s)
    offsets = torch.empty(B * (XYZ + 1), dtype=torch.int32, device=device)
    order = torch.empty(B * P, dtype=torch.int32, device=device)
    tiles = torch.empty(B * _lib.call_raw("e2ep_lss_tiles", XYZ), dtype=torch.int32, device=device)
    ws = torch.empty(B * XYZ, dtype=torch.int32, device=device)
    _lib.call("e2ep_lss_plan", _lib.ptr(pillar), B, N, D, h, w, XYZ, _lib.ptr(offsets),
              _lib.ptr(order), _lib.ptr(tiles), _lib.ptr(ws), _lib.nbytes(ws), s)
    return LssPlan(pillar, offsets, order, tiles, B, N, D, h, w, X, Y, Z)


def transpose(x, rows, cols, batch, in_bstride=None):
    """out[b, c, r] = x[b, r, c] for a (batch, rows, cols) view with batch stride in_bstride."""
    out = torch.empty(batch, cols, rows, dtype=torch.float32, device=x.device)
    _lib.call("e2ep_transpose", _lib.ptr(x), rows * cols if in_bstride is None else in_bstride,
              batch, rows, cols, _lib.ptr(out), _lib.stream())
    return out


class _LiftSplat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prob, feat, plan, out_channels):
        p = plan
        BN, C = feat.shape[0], feat.shape[1]
        hw = p.h * p.w
        prob = prob.contiguous()
        featT = transpose(feat.contiguous(), C, hw, BN)           # (B*N, hw, C)
        out = torch.empty(p.B, out_channels, p.X, p.Y, dtype=torch.float32, device=feat.device)
        with timing.region("lss_fwd"):
            _lib.call("e2ep_lss_fwd", _lib.ptr(prob), _lib.ptr(featT), _lib.ptr(p.offsets),
                      _lib.ptr(p.order), _lib.ptr(p.tiles), p.B, p.N, p.D, hw, C, p.XYZ, _lib.ptr(out),
                      out_channels * p.XYZ, _lib.stream())
        ctx.save_for_backward(prob, featT)
        ctx.plan, ctx.C = plan, C
        return out

    @staticmethod
    def backward(ctx, gout):
        prob, featT = ctx.saved_tensors
        p, C = ctx.plan, ctx.C
        hw = p.h * p.w
        if gout.shape[1] == C and gout.is_contiguous(memory_format=torch.channels_last):
            gT = gout  # pillar-major already (the BEV stem's resize backward writes it so)
        else:
            gout = gout.contiguous()
            gT = transpose(gout, C, p.XYZ, p.B, in_bstride=gout.shape[1] * p.XYZ)  # (B, XYZ, C)
        gp = torch.empty_like(prob)
        gf = torch.empty(p.B * p.N, C, p.h, p.w, dtype=torch.float32, device=gout.device)
        with timing.region("lss_bwd"):
            _lib.call("e2ep_lss_bwd", _lib.ptr(gT), _lib.ptr(prob), _lib.ptr(featT),
                      _lib.ptr(p.pillar), p.B, p.N, p.D, hw, C, p.XYZ, _lib.ptr(gp), _lib.ptr(gf),
                      _lib.stream())
        return gp, gf, None, None


def lift_splat(prob, feat, plan, out_channels=None):
    """Pool prob (B*N,D,h,w) x feat (B*N,C,h,w) into a (B, out_channels, X, Y) BEV tensor.

    Channels [0, C) hold the pooled features (every cell written); channels [C, out_channels)
    are left for the caller to fill (e.g. the target-point channel)."""
    _require_device(prob, feat)
    C = feat.shape[1]
    return _LiftSplat.apply(prob, feat, plan, C if out_channels is None else out_channels)


def target_bev(out, channel, target_point, noise, res_x, res_y):
    """Write the target-point plane into out[:, channel] (model/parking_model.py:28-46)."""
    _require_device(out)
    B, Ctot, X, Y = out.shape
    tp = target_point.to(device=out.device, dtype=torch.float32).contiguous()
    nz = noise.to(device=out.device, dtype=torch.float32).contiguous()
    plane = out[:, channel]
    _lib.call("e2ep_target_bev", _lib.ptr(tp), _lib.ptr(nz), B, X, Y, float(res_x), float(res_y),
              _lib.ptr(plane), Ctot * X * Y, _lib.stream())
    return out
