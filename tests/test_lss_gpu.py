"""Lift-splat HIP kernels vs the oracle / golden vectors (MI355X)."""
import hashlib

import numpy as np
import pytest
import torch

from helpers import golden, max_scaled, meta, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plan_from_golden(g, B=1, lo=None, res=None):
    from e2ep_amd import lss
    g4 = golden("geometry_4cam_256.npz")
    comb = torch.from_numpy(g["combine"])[None].expand(B, -1, -1, -1).contiguous()
    trans = torch.from_numpy(g["trans"])[None].expand(B, -1, -1).contiguous()
    return lss.build_plan(torch.from_numpy(g["frustum"]), comb, trans, g4["lo"].tolist(),
                          g4["res"].tolist(), g4["dim"].tolist(), DEV)


def test_pillar_index_bit_exact_4cam():
    g = golden("geometry_4cam_256.npz")
    plan = _plan_from_golden(g)
    got = plan.pillar.view(g["pillar"].shape).cpu().numpy()
    assert np.array_equal(got, g["pillar"])


def test_pillar_index_bit_exact_hires_6cam():
    g = golden("geometry_6cam_512.npz")
    plan = _plan_from_golden(g)
    got = plan.pillar.cpu().numpy().astype(np.int32)
    assert hashlib.sha256(got.tobytes()).hexdigest() == meta()["geometry_6cam_512"]["pillar_sha256"]


def _pillar_from_rig(K, E, frustum):
    from e2ep_amd import lss
    g4 = golden("geometry_4cam_256.npz")
    comb, trans = lss.rig_transforms(K[None], E[None], DEV)
    plan = lss.build_plan(torch.from_numpy(frustum), comb, trans, g4["lo"].tolist(), g4["res"].tolist(),
                          g4["dim"].tolist(), DEV)
    return comb[0].cpu().numpy(), plan.pillar.cpu().numpy().astype(np.int32)


def test_device_rig_algebra_reproduces_reference_pillars_4cam():
    """End to end from K,E: the device rig algebra (fp64, deterministic) lands within a few ulp (fp32 LU error, measured 11) of
    the reference's fp32 LAPACK combine and gives the reference's pillar table bit for bit."""
    g = golden("geometry_4cam_256.npz")
    comb, pil = _pillar_from_rig(torch.from_numpy(g["K"]), torch.from_numpy(g["E"]), g["frustum"])
    ulp = np.abs(comb.view(np.int32).astype(np.int64) - g["combine"].view(np.int32).astype(np.int64))
    assert ulp[np.abs(g["combine"]) > 1e-6].max() <= 16  # fp32 LU vs fp64 GJ: measured 11
    assert np.array_equal(pil, g["pillar"].reshape(-1))


def test_device_rig_algebra_hires_6cam_band():
    """The device rig algebra entry point (e2ep_rig_transforms, lss.rig_transforms: fp64
    Gauss-Jordan on the GPU) vs the reference's fp32 LAPACK combine at 6-cam 512^2.  LAPACK's
    last ulp is not reproducible on the device and a handful of the 1.18M points sit within an
    ulp of a cell edge; the flip count is recorded.  No product path plans with it since round
    6 — a captured step reuses a plan built with the reference's fp32 host algebra before the
    capture (test_captured_device_rig_plan_bit_exact_c4) — so every product path is bit-exact
    (0 flips)."""
    from test_model_b8_gpu import _record
    g = golden("geometry_6cam_512.npz")
    from oracle import geom_c
    g4 = golden("geometry_4cam_256.npz")
    ref = geom_c.geom_index(g["frustum"], g["combine"], g["trans"], g4["lo"], g4["res"], g4["dim"]).reshape(-1)
    _, pil = _pillar_from_rig(torch.from_numpy(g["K"]), torch.from_numpy(g["E"]), g["frustum"])
    flips = int((pil != ref).sum())
    print(f"capture-path device-rig pillar flips at 6x512^2: {flips} of {pil.size}")
    _record("rig", "capture_fp64_device_algebra_6cam_flips", flips=flips, points=int(pil.size))
    assert flips <= 16


@pytest.mark.parametrize("rig", ["geometry_4cam_256.npz", "geometry_6cam_512.npz"])
def test_device_rig_pillar_index_bit_exact_end_to_end(rig):
    """K, E already on the GPU through BevModel.plan (outside a capture): the rig is copied to
    the host and goes through the reference's own fp32 CPU algebra, so the pillar table equals
    the reference golden bit for bit (0 flips) at both rigs, at B=1 and over a B=4 batch."""
    from model.bev_model import BevModel
    from tool.config import default_cfg
    g = golden(rig)
    hires = "6cam" in rig
    cfg = default_cfg(final_dim=[512, 512], image_crop=512) if hires else default_cfg()
    bm = BevModel(cfg).to(DEV)
    for B in (1, 4):
        K = torch.from_numpy(g["K"])[None].repeat(B, 1, 1, 1).to(DEV)
        E = torch.from_numpy(g["E"])[None].repeat(B, 1, 1, 1).to(DEV)
        pil = bm.plan(K, E, DEV).pillar.view(B, -1).cpu().numpy().astype(np.int32)
        for b in range(B):
            if hires:
                ref = meta()["geometry_6cam_512"]["pillar_sha256"]
                assert hashlib.sha256(pil[b].tobytes()).hexdigest() == ref
            else:
                flips = int((pil[b] != g["pillar"].reshape(-1)).sum())
                assert flips == 0, flips


def test_captured_device_rig_plan_bit_exact_c4(monkeypatch):
    """C4 (6 x 512^2, B = 4) with the rig on the GPU inside a HIP-graph capture (reference
    model/bev_model.py:45-57,85-96): the capture reuses the plan BevModel.plan built outside it
    with the reference's fp32 host algebra — the same plan object, its pillar table equal to
    the reference golden for every sample (0 flips, recorded) — and the captured lift-splat
    replays bitwise what the eager call computes.  A device rig met first inside a capture
    raises instead of planning with the device algebra."""
    from e2ep_amd import _lib, graphs, lss
    from model.bev_model import BevModel
    from test_model_b8_gpu import _record
    from tool.config import default_cfg
    g = golden("geometry_6cam_512.npz")
    bm = BevModel(default_cfg(final_dim=[512, 512], image_crop=512)).to(DEV)
    B = 4
    K = torch.from_numpy(g["K"])[None].repeat(B, 1, 1, 1).to(DEV)
    E = torch.from_numpy(g["E"])[None].repeat(B, 1, 1, 1).to(DEV)
    with monkeypatch.context() as mp_:  # the capture branch, without a real capture
        mp_.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
        with pytest.raises(_lib.E2EPError, match="before the capture"):
            bm.plan(K, E, DEV)
    plan = bm.plan(K, E, DEV)  # outside the capture: host algebra, pinned for the capture
    N, D, hw = 6, 48, 64 * 64
    gl = torch.Generator().manual_seed(3)
    prob = torch.rand(B * N, D, 64, 64, generator=gl).to(DEV)
    feat = torch.randn(B * N, 64, 64, 64, generator=gl).to(DEV)
    seen = []

    def body():
        p = bm.plan(K, E, DEV)
        seen.append(p)
        return lss.lift_splat(prob, feat, p)

    want = body().clone()
    graph, out, _ = graphs.capture(body)
    graph.replay()
    torch.cuda.synchronize()
    assert seen[-1] is plan and seen[0] is plan
    assert torch.equal(out, want)
    pil = plan.pillar.view(B, -1).cpu().numpy().astype(np.int32)
    ref = meta()["geometry_6cam_512"]["pillar_sha256"]
    flips = sum(hashlib.sha256(pil[b].tobytes()).hexdigest() != ref for b in range(B))
    _record("rig", "captured_device_rig_c4_b4_samples_off_golden", flips=int(flips), samples=B)
    assert flips == 0


@pytest.mark.parametrize("rig", ["geometry_4cam_256.npz", "geometry_6cam_512.npz"])
def test_host_rig_pillar_index_bit_exact_end_to_end(rig):
    """From K, E as the data loader delivers them (host tensors) through BevModel.plan — the
    product path of every train / predict step: the rig algebra is the reference's own fp32 CPU
    ops (model/bev_model.py:46-53) and the pillar table equals the reference golden bit for
    bit at both rigs (0 flips), at B=1 and replicated over a B=4 batch."""
    from model.bev_model import BevModel
    from tool.config import default_cfg
    g = golden(rig)
    hires = "6cam" in rig
    cfg = default_cfg(final_dim=[512, 512], image_crop=512) if hires else default_cfg()
    bm = BevModel(cfg).to(DEV)
    assert np.array_equal(bm.frustum.detach().cpu().numpy(), g["frustum"])
    for B in (1, 4):
        K = torch.from_numpy(g["K"])[None].repeat(B, 1, 1, 1)
        E = torch.from_numpy(g["E"])[None].repeat(B, 1, 1, 1)
        pil = bm.plan(K, E, DEV).pillar.view(B, -1).cpu().numpy().astype(np.int32)
        for b in range(B):
            if hires:  # the golden stores the table's hash
                assert hashlib.sha256(pil[b].tobytes()).hexdigest() == \
                    meta()["geometry_6cam_512"]["pillar_sha256"]
            else:
                assert np.array_equal(pil[b], g["pillar"].reshape(-1))


def test_plan_invariants_batch_of_different_rigs():
    """Counting sort: per-pillar counts, ascending codes within a pillar, every kept point once."""
    from e2ep_amd import lss, synthetic
    g4 = golden("geometry_4cam_256.npz")
    K, E = synthetic.rig()
    E2 = E.clone()
    E2[:, :3, 3] += torch.tensor([0.13, -0.07, 0.02])  # second sample: shifted rig
    comb, trans = lss.rig_transforms(torch.stack([K, K]), torch.stack([E, E2]), DEV)
    plan = lss.build_plan(torch.from_numpy(g4["frustum"]), comb, trans, g4["lo"].tolist(),
                          g4["res"].tolist(), [200, 200, 1], DEV)
    pil = plan.pillar.view(2, -1).cpu().numpy()
    off = plan.offsets.view(2, -1).cpu().numpy()
    order = plan.order.view(2, -1).cpu().numpy()
    P = pil.shape[1]
    for b in range(2):
        kept = pil[b][pil[b] >= 0]
        cnt = np.bincount(kept, minlength=40000)
        assert np.array_equal(np.diff(off[b]), cnt)
        codes = order[b][: off[b][-1]]
        n, d, pix = codes >> 24, (codes >> 16) & 255, codes & 65535
        flat = n * (48 * 1024) + d * 1024 + pix
        assert np.array_equal(np.sort(flat), np.nonzero(pil[b] >= 0)[0])
        assert np.array_equal(pil[b][flat], np.repeat(np.arange(40000), cnt))
        for q in np.nonzero(cnt > 1)[0][:2000]:
            seg = codes[off[b][q]:off[b][q + 1]]
            assert np.all(np.diff(seg) > 0)
    assert not np.array_equal(pil[0], pil[1])
    # forward tile schedule at B = 2 (lane schedule, include/e2ep.h): 8 lanes; lane l holds
    # pillar range g = l // 2 of sample l % 2: G = 4 contiguous ranges per sample that cover
    # every tile once, with point-balanced boundaries (a tile belongs to the range its point
    # midpoint falls in) of at most L = ceil(1.5 ceil(nt / G)) tiles, heaviest first (ties by
    # index), -1 padded
    T, B, G = 64, 2, 4
    nt = -(-40000 // T)
    L = -(-3 * -(-nt // G) // 2)
    lanes = plan.tiles.cpu().numpy()[:8 * L].reshape(8, L)
    for b in range(B):
        edges = np.minimum(np.arange(nt + 1) * T, 40000)
        cnt = off[b][edges[1:]] - off[b][edges[:-1]]
        before = off[b][edges[:-1]] - off[b][0]
        total = int(off[b][-1] - off[b][0])
        rng = np.minimum(G - 1, ((2 * before + cnt) * G) // (2 * total))
        bnd = np.searchsorted(rng, np.arange(G + 1), side="left")
        even = np.diff(bnd).max() > L
        if even:
            bnd = -(-np.arange(G + 1) * nt // G)  # the even cut
        seen = []
        for g in range(G):
            lo, hi = bnd[g], bnd[g + 1]
            lane = lanes[g * B + b]
            want = lo + np.lexsort((np.arange(hi - lo), -cnt[lo:hi]))
            assert np.array_equal(lane[:hi - lo], want)
            assert np.all(lane[hi - lo:] == -1)
            seen.extend(lane[:hi - lo])
            # balanced: a range's points within one tile of the even share
            assert even or abs(int(cnt[lo:hi].sum()) - total / G) <= cnt.max()
        assert np.array_equal(np.sort(seen), np.arange(nt))


def test_lss_fwd_schedule_does_not_change_result():
    """Any tile order gives the bitwise-same BEV (each pillar's sum order is fixed); the
    natural order (tiles=NULL) vs the scheduled order (heaviest-first per sample at B = 3 / 8,
    the XCD lane schedule at B = 1 / 2 / 4), C=64 and the C%4!=0 path; every cell written."""
    g = golden("geometry_4cam_256.npz")
    for B in (1, 2, 3, 4, 8):  # lane schedules (1, 2, 4), per-sample order (3, 8)
        _schedule_case(B, g)


def _schedule_case(B, g):
    from e2ep_amd import _lib
    N, D, hw = 4, 48, 1024
    plan = _plan_from_golden(g, B)
    gl = torch.Generator().manual_seed(5 + B)
    prob = torch.rand(B * N, D, hw, generator=gl).to(DEV)
    for C in (64, 12, 6):
        featT = torch.randn(B * N, hw, C, generator=gl).to(DEV)
        outs = []
        for tiles in (plan.tiles, None):
            bev = torch.full((B, C, 40000), float("nan"), device=DEV)
            _lib.call("e2ep_lss_fwd", _lib.ptr(prob), _lib.ptr(featT), _lib.ptr(plan.offsets),
                      _lib.ptr(plan.order), _lib.ptr(tiles), B, N, D, hw, C, 40000, _lib.ptr(bev),
                      C * 40000, _lib.stream())
            outs.append(bev.cpu())
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[0], outs[1])


def _lss_inputs(m):
    B, N, D, h, w, C = m["shape"]
    gl = torch.Generator().manual_seed(m["seed"])
    logits = torch.randn(B * N, D, h, w, generator=gl) * m["logit_scale"]
    feat = torch.randn(B * N, C, h, w, generator=gl)
    gout = torch.randn(B, C, 200, 200, generator=gl)
    return logits.softmax(1), feat, gout


def test_lss_fwd_bwd_matches_reference_golden():
    """Reference VoxelsSumming path (golden) vs fused HIP kernel at C=4.  Tolerances follow
    SURVEY.md §8c: the reference's own cumsum trick carries ~1e-6 abs noise."""
    from e2ep_amd import lss
    g = golden("geometry_4cam_256.npz")
    ref = golden("lss_c4.npz")
    prob, feat, gout = _lss_inputs(meta()["lss_c4"])
    plan = _plan_from_golden(g)
    p = prob.to(DEV).requires_grad_(True)
    f = feat.to(DEV).requires_grad_(True)
    bev = lss.lift_splat(p, f, plan)
    bev.backward(gout.to(DEV))
    assert max_scaled(bev, ref["bev"]) < 1e-4 and rel_l2(bev, ref["bev"]) < 1e-4
    assert rel_l2(p.grad, ref["grad_prob"]) < 1e-5
    assert rel_l2(f.grad, ref["grad_feat"]) < 1e-5


def test_lss_full_channels_vs_oracle_and_determinism():
    """C=64 (product width), B=2: HIP vs the oracle's reference-order splat; bitwise repeatable."""
    from e2ep_amd import lss
    from oracle import parking_ref as O
    g = golden("geometry_4cam_256.npz")
    B, N, D, h, w, C = 2, 4, 48, 32, 32, 64
    gl = torch.Generator().manual_seed(11)
    prob = (torch.randn(B * N, D, h, w, generator=gl) * 3).softmax(1)
    feat = torch.randn(B * N, C, h, w, generator=gl)
    gout = torch.randn(B, C + 1, 200, 200, generator=gl)
    plan = _plan_from_golden(g, B)
    outs = []
    for _ in range(2):
        p = prob.to(DEV).requires_grad_(True)
        f = feat.to(DEV).requires_grad_(True)
        bev = lss.lift_splat(p, f, plan, C + 1)
        bev[:, C].zero_()
        bev.backward(gout.to(DEV))
        outs.append((bev[:, :C].detach().cpu(), p.grad.cpu(), f.grad.cpu()))
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1])), "not run-to-run deterministic"
    po = prob.clone().requires_grad_(True)
    fo = feat.clone().requires_grad_(True)
    outer = (po.unsqueeze(1) * fo.unsqueeze(2)).view(B, N, C, D, h, w).permute(0, 1, 3, 4, 5, 2)
    xyz = torch.from_numpy(g["xyz"])[None].expand(B, -1, -1, -1, -1, -1)
    res = torch.from_numpy(g["res"])
    ref = O.splat(xyz, outer, res, torch.from_numpy(g["lo"]) + res / 2.0, torch.from_numpy(g["dim"]))
    ref.backward(gout[:, :C])
    bev, gp, gf = outs[0]
    assert max_scaled(bev, ref) < 1e-4 and rel_l2(bev, ref) < 1e-4
    assert rel_l2(gp, po.grad) < 1e-5 and rel_l2(gf, fo.grad) < 1e-5
    # against an exact fp64 segmented sum the direct per-pillar sum is far tighter than the
    # reference's cumsum-difference
    pil = torch.from_numpy(g["pillar"]).reshape(-1).long()
    keep = pil >= 0
    exact = torch.zeros(B, 40000, C, dtype=torch.float64)
    for b in range(B):
        pts = (prob[b * N:(b + 1) * N].double().permute(0, 2, 3, 1).unsqueeze(-1)
               * feat[b * N:(b + 1) * N].double().permute(0, 2, 3, 1).unsqueeze(-2))  # n,h,w,D,C
        pts = pts.permute(0, 3, 1, 2, 4).reshape(-1, C)
        exact[b].index_add_(0, pil[keep], pts[keep])
    exact = exact.permute(0, 2, 1).reshape(B, C, 200, 200)
    assert rel_l2(bev, exact) < 5e-7 and rel_l2(ref, exact) > rel_l2(bev, exact)
    # cells no point falls in are exactly zero, as in the reference
    occ = torch.bincount(torch.from_numpy(g["pillar"]).reshape(-1).long().clamp(min=0)[
        torch.from_numpy(g["pillar"]).reshape(-1) >= 0], minlength=40000).view(200, 200) > 0
    empty = ~occ
    assert torch.count_nonzero(bev[:, :, empty]) == 0 and torch.count_nonzero(ref[:, :, empty]) == 0


@pytest.mark.parametrize("xy", [(1.23, -2.71), (9.8, 9.9), (-9.97, -9.6), (-12.0, 3.0), (15.0, -15.0),
                                (0.0, 0.0), (-10.4, -10.45), (-11.0, 5.0)])
def test_target_bev_matches_reference_semantics(xy):
    from e2ep_amd import lss
    from oracle import parking_ref as O
    B = 3
    tp = torch.tensor([[xy[0], xy[1], 30.0]] * B)
    noise = torch.tensor([[0.0, 0.999], [0.5, 0.05], [0.93, 0.41]])
    m = O.ParkingModelRef.__new__(O.ParkingModelRef)
    m.cfg = O.Cfg
    _, ref = O.ParkingModelRef.add_target_bev(m, torch.zeros(B, 2, 200, 200), tp, noise)
    out = torch.full((B, 3, 200, 200), 7.0, device=DEV)
    lss.target_bev(out, 2, tp, noise, 0.1, 0.1)
    assert torch.equal(out[:, 2:].cpu(), ref)
    assert (out[:, :2] == 7.0).all()


def test_lss_hires_6cam_512_vs_fp64():
    """C4 geometry (6 cams, 512^2 images -> 64x64 feature grid, 1.18 M points per sample,
    up to 414 per pillar), C=64: fused forward / backward vs exact fp64 segment sums over the
    oracle's (C restatement's) pillar table."""
    from e2ep_amd import lss
    from oracle import geom_c
    g = golden("geometry_6cam_512.npz")
    g4 = golden("geometry_4cam_256.npz")
    N, D, h, w, C = 6, 48, 64, 64, 64
    pil = torch.from_numpy(geom_c.geom_index(g["frustum"], g["combine"], g["trans"], g4["lo"],
                                             g4["res"], g4["dim"]).reshape(N, D * h * w)).long()
    plan = _plan_from_golden(g)
    gl = torch.Generator().manual_seed(21)
    prob = (torch.randn(N, D, h, w, generator=gl) * 2).softmax(1)
    feat = torch.randn(N, C, h, w, generator=gl)
    gout = torch.randn(1, C, 200, 200, generator=gl)
    p = prob.to(DEV).requires_grad_(True)
    f = feat.to(DEV).requires_grad_(True)
    bev = lss.lift_splat(p, f, plan)
    bev.backward(gout.to(DEV))
    exact = torch.zeros(40000, C, dtype=torch.float64)
    G = gout[0].reshape(C, 40000).double().t()  # (XY, C)
    gp_ref = torch.zeros(N, D * h * w, dtype=torch.float64)
    gf_ref = torch.zeros(N, h * w, C, dtype=torch.float64)
    for n in range(N):
        keep = pil[n] >= 0
        q = pil[n][keep]
        pr = prob[n].reshape(D, h * w).double()  # (D, hw)
        ft = feat[n].reshape(C, h * w).double().t()  # (hw, C)
        idx = torch.nonzero(keep).squeeze(1)
        d, pix = idx // (h * w), idx % (h * w)
        pts = pr[d, pix].unsqueeze(1) * ft[pix]  # (kept, C)
        exact.index_add_(0, q, pts)
        gq = G[q]  # (kept, C)
        gp_ref[n, idx] = (gq * ft[pix]).sum(1)
        gf_ref[n].index_add_(0, pix, pr[d, pix].unsqueeze(1) * gq)
    ref = exact.t().reshape(1, C, 200, 200)
    assert rel_l2(bev, ref) < 1e-5 and max_scaled(bev, ref) < 1e-5
    assert rel_l2(p.grad.reshape(N, -1), gp_ref) < 1e-5
    assert rel_l2(f.grad.reshape(N, C, h * w).transpose(1, 2), gf_ref) < 1e-5


def test_lss_plan_refuses_short_workspace():
    """e2ep_lss_plan checks workspace_bytes against e2ep_lss_plan_workspace (ABI 4)."""
    from e2ep_amd import _lib
    B, N, D, h, w, XYZ = 1, 4, 48, 32, 32, 40000
    P = N * D * h * w
    pillar = torch.full((B * P,), -1, dtype=torch.int32, device=DEV)
    offsets = torch.empty(B * (XYZ + 1), dtype=torch.int32, device=DEV)
    order = torch.empty(B * P, dtype=torch.int32, device=DEV)
    need = _lib.call_raw("e2ep_lss_plan_workspace", B, XYZ)
    ws = torch.empty(need // 4, dtype=torch.int32, device=DEV)
    with pytest.raises(_lib.E2EPError, match="workspace"):
        _lib.call("e2ep_lss_plan", _lib.ptr(pillar), B, N, D, h, w, XYZ, _lib.ptr(offsets),
                  _lib.ptr(order), None, _lib.ptr(ws), need - 4, _lib.stream())
    _lib.call("e2ep_lss_plan", _lib.ptr(pillar), B, N, D, h, w, XYZ, _lib.ptr(offsets),
              _lib.ptr(order), None, _lib.ptr(ws), need, _lib.stream())
    torch.cuda.synchronize()
    assert int(offsets[-1]) == 0
