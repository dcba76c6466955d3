"""k_conv_stem_lp / k_conv_stem_dgrad_lp (csrc/conv_stem.hip): the direct-convolution forward
and data gradient of 7x7 / 2 convs with 64 output channels on 16-bit operands — the BEV stem
(reference model/bev_encoder.py:13,26) in C3 (bf16) and C5 (fp16).  Against fp64 convolutions
of the operands rounded to the 16-bit format (the products are exact, the sums fp32), against
the implicit-GEMM kernel they replace (k_conv_lp, e2ep_tune key 35 = 1: same rounding, another
fp32 sum order), and run to run bitwise.  Key 35 = 1 + mask (1 forward, 2 data gradient, 4 weight
gradient, k_conv_stem_wgrad_lp, bf16 only)."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
KEY = 35  # tune.h TUNE_STEM_DIRECT

# (N, Cin, H, W, bias, act): Cin % 16 = remainder channels on the flattened tail steps
CASES = [
    (2, 65, 256, 256, False, 0),  # the BEV stem at full size (4 tail steps)
    (2, 65, 50, 70, False, 0),    # ragged output tiles (25 x 35)
    (1, 64, 64, 64, False, 0),    # no remainder
    (2, 3, 40, 36, False, 0),     # remainder only (no 16-channel chunk)
    (1, 68, 32, 48, False, 0),    # 4 remainder channels (14 tail steps, the cap)
    (2, 65, 64, 64, True, 1),     # bias + relu epilogue
    (2, 21, 30, 30, False, 0),    # 5 remainder channels: stays on k_conv_lp
]


def _run(x, w, b, act, mode, key):
    from e2ep_amd import _lib, conv, precision
    old = _lib.call_raw("e2ep_tune", KEY, key)
    try:
        with precision.use(mode):
            return conv.conv2d(x, w, b, (2, 2), (3, 3, 3, 3), (1, 1), act)
    finally:
        _lib.call_raw("e2ep_tune", KEY, old)


@pytest.mark.parametrize("mode,dt", [("bf16", torch.bfloat16), ("fp16", torch.float16)])
@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_stem_direct_vs_rounded_fp64(case, mode, dt):
    N, Cin, H, W, has_b, act = case
    if mode == "fp16" and N * H * W > 40000:
        pytest.skip("fp16 covered at the smaller shapes")
    g = torch.Generator().manual_seed(7 + Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(64, Cin, 7, 7, generator=g) / (Cin * 49) ** 0.5
    b = torch.randn(64, generator=g) if has_b else None
    xd, wd = x.to(DEV), w.to(DEV)
    bd = b.to(DEV) if has_b else None
    with torch.no_grad():
        y = _run(xd, wd, bd, act, mode, 2)
        y2 = _run(xd, wd, bd, act, mode, 2)
        y_gemm = _run(xd, wd, bd, act, mode, 1)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)  # deterministic
    r = lambda t: t.to(dt).double()  # noqa: E731
    ref = F.conv2d(r(x), r(w), b.double() if has_b else None, 2, 3)
    if act:
        ref = ref.clamp_min(0)
    assert y.shape == ref.shape
    assert rel_l2(y, ref) < 2e-6
    assert rel_l2(y, y_gemm) < 2e-6
    assert (y.cpu().double() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


# (N, Cin, H, W): the data gradient into the first 64 input channels (pad 3)
DG_CASES = [
    (2, 65, 256, 256),  # the BEV stem at full size
    (2, 65, 50, 70),    # ragged coarse tiles
    (1, 64, 64, 64),    # every input channel
    (1, 65, 33, 47),    # odd sizes: the last phase row / column partly outside
]


@pytest.mark.parametrize("mode,dt", [("bf16", torch.bfloat16), ("fp16", torch.float16)])
@pytest.mark.parametrize("case", DG_CASES, ids=[str(i) for i in range(len(DG_CASES))])
def test_stem_direct_dgrad_vs_rounded_fp64(case, mode, dt):
    from e2ep_amd import _lib, conv, precision
    N, Cin, H, W = case
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dims = (N, Cin, H, W, 64, 7, 7, P, Q, 2, 2, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(5 + H + W)
    w = torch.randn(64, Cin, 7, 7, generator=g) / (Cin * 49) ** 0.5
    gy = torch.randn(N, 64, P, Q, generator=g)
    wt = conv.tap_major(w.to(DEV))
    gyd = gy.to(DEV)
    out = {}
    for key in (4, 1):
        old = _lib.call_raw("e2ep_tune", KEY, key)
        try:
            with precision.use(mode):
                for rep in range(2 if key == 4 else 1):
                    dx = torch.empty(N, 64, H, W, device=DEV)
                    conv.conv_dgrad(gyd, wt, dims, 64, dx, w_layout=1)
                    out[(key, rep)] = dx
        finally:
            _lib.call_raw("e2ep_tune", KEY, old)
    torch.cuda.synchronize()
    assert torch.equal(out[(4, 0)], out[(4, 1)])  # deterministic
    r = lambda t: t.to(dt).double()  # noqa: E731
    x64 = torch.zeros(N, Cin, H, W, dtype=torch.float64, requires_grad=True)
    F.conv2d(x64, r(w), None, 2, 3).backward(r(gy))
    ref = x64.grad[:, :64]
    assert rel_l2(out[(4, 0)], ref) < 2e-6
    assert rel_l2(out[(4, 0)], out[(1, 0)]) < 2e-6
    assert (out[(4, 0)].cpu().double() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


def test_stem_direct_in_bev_stem_training_step():
    """The BEV stem op (bev_stem: resize + conv) in C3 on the direct kernels (key 35 = 8) against
    the implicit-GEMM kernels (key 35 = 1): the output and both gradients agree to fp32 sum
    order."""
    from e2ep_amd import _lib, bev_stem, precision
    g = torch.Generator().manual_seed(11)
    bev = torch.randn(2, 64, 200, 200, generator=g).to(DEV)
    tgt = torch.randn(2, 1, 200, 200, generator=g).to(DEV)
    w = (torch.randn(64, 65, 7, 7, generator=g) / 22.6).to(DEV)
    gy = torch.randn(2, 64, 128, 128, generator=g).to(DEV)
    out = {}
    for key in (8, 1):
        old = _lib.call_raw("e2ep_tune", KEY, key)
        try:
            b = bev.clone().requires_grad_(True)
            wd = w.clone().requires_grad_(True)
            with precision.use("bf16"):
                y = bev_stem.bev_stem(b, tgt, wd, (256, 256))
                y.backward(gy)
            out[key] = (y.detach(), b.grad, wd.grad)
        finally:
            _lib.call_raw("e2ep_tune", KEY, old)
    assert rel_l2(out[8][0], out[1][0]) < 2e-6
    assert rel_l2(out[8][1], out[1][1]) < 2e-6
    assert rel_l2(out[8][2], out[1][2]) < 2e-6


# (N, Cin, H, W): weight gradient, Q % 8 == 0
WG_CASES = [
    (2, 65, 256, 256),  # the BEV stem at full size (9 channel chunks, the last one channel)
    (2, 65, 50, 80),    # ragged row tiles (P = 25), Q = 40
    (1, 64, 64, 64),    # whole chunks
    (1, 3, 32, 48),     # one partial chunk
    (3, 17, 40, 16),    # Q = 8: one octet of a 32-column tile
]


@pytest.mark.parametrize("case", WG_CASES, ids=[str(i) for i in range(len(WG_CASES))])
def test_stem_direct_wgrad_vs_rounded_fp64(case):
    from e2ep_amd import _lib, conv, precision
    N, Cin, H, W = case
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dims = (N, Cin, H, W, 64, 7, 7, P, Q, 2, 2, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(9 + H + W + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    gy = torch.randn(N, 64, P, Q, generator=g)
    xd, gyd = x.to(DEV), gy.to(DEV)
    out = {}
    for key in (8, 1):
        old = _lib.call_raw("e2ep_tune", KEY, key)
        try:
            with precision.use("bf16"):
                for rep in range(2 if key == 8 else 1):
                    dw = torch.empty(64, Cin, 7, 7, device=DEV)
                    conv.conv_wgrad(gyd, xd, dims, dw)
                    out[(key, rep)] = dw
        finally:
            _lib.call_raw("e2ep_tune", KEY, old)
    torch.cuda.synchronize()
    assert torch.equal(out[(8, 0)], out[(8, 1)])  # deterministic
    r = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    w64 = torch.zeros(64, Cin, 7, 7, dtype=torch.float64, requires_grad=True)
    F.conv2d(r(x), w64, None, 2, 3).backward(r(gy))
    assert rel_l2(out[(8, 0)], w64.grad) < 5e-6
    assert rel_l2(out[(8, 0)], out[(1, 0)]) < 5e-6


# fp32 operands (C2, exact-f32 MFMA, key 35 mask 8 gradients / 16 forward): the same kernels with
# v_mfma_f32_32x32x2_f32
F32_CASES = [(2, 65, 256, 256), (2, 65, 50, 70), (1, 64, 64, 64), (1, 68, 32, 48)]


@pytest.mark.parametrize("case", F32_CASES, ids=[str(i) for i in range(len(F32_CASES))])
def test_stem_direct_fp32_vs_fp64(case):
    from e2ep_amd import _lib, conv
    N, Cin, H, W = case
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dims = (N, Cin, H, W, 64, 7, 7, P, Q, 2, 2, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(13 + H + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(64, Cin, 7, 7, generator=g) / (Cin * 49) ** 0.5
    gy = torch.randn(N, 64, P, Q, generator=g)
    xd, wd, gyd = x.to(DEV), w.to(DEV), gy.to(DEV)
    wt = conv.tap_major(wd)
    out = {}
    for key in (28, 1):
        old = _lib.call_raw("e2ep_tune", KEY, key)
        try:
            with torch.no_grad():
                y = conv.conv2d(xd, wd, None, (2, 2), (3, 3, 3, 3), (1, 1), 0)
            dx = torch.empty(N, 64, H, W, device=DEV)
            conv.conv_dgrad(gyd, wt, dims, 64, dx, w_layout=1)
            out[key] = (y, dx)
        finally:
            _lib.call_raw("e2ep_tune", KEY, old)
    torch.cuda.synchronize()
    y64 = F.conv2d(x.double(), w.double(), None, 2, 3)
    x64 = torch.zeros(N, Cin, H, W, dtype=torch.float64, requires_grad=True)
    F.conv2d(x64, w.double(), None, 2, 3).backward(gy.double())
    # fp32 sums of up to 65 x 49 products in another order than k_conv_gemm2's: ~1e-6
    # relative (test_conv_gpu.py holds the implicit GEMMs to 1e-5 against fp64)
    assert rel_l2(out[28][0], y64) < 5e-6
    assert rel_l2(out[28][1], x64.grad[:, :64]) < 5e-6
    assert rel_l2(out[28][0], out[1][0]) < 5e-6
    assert rel_l2(out[28][1], out[1][1]) < 5e-6


@pytest.mark.parametrize("case", WG_CASES, ids=[str(i) for i in range(len(WG_CASES))])
def test_stem_direct_wgrad_fp32_vs_fp64(case):
    """k_conv_stem_wgrad_lp<0> (exact-f32 MFMA, key 35 mask 4 | 8): C2's stem weight gradient,
    and C5's (its fp16 mode keeps the weight gradient fp32)."""
    from e2ep_amd import _lib, conv
    N, Cin, H, W = case
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dims = (N, Cin, H, W, 64, 7, 7, P, Q, 2, 2, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(17 + H + W + Cin)
    x = torch.randn(N, Cin, H, W, generator=g)
    gy = torch.randn(N, 64, P, Q, generator=g)
    xd, gyd = x.to(DEV), gy.to(DEV)
    out = {}
    for key in (16, 1):
        old = _lib.call_raw("e2ep_tune", KEY, key)
        try:
            dw = torch.empty(64, Cin, 7, 7, device=DEV)
            conv.conv_wgrad(gyd, xd, dims, dw)
            out[key] = dw
        finally:
            _lib.call_raw("e2ep_tune", KEY, old)
    torch.cuda.synchronize()
    w64 = torch.zeros(64, Cin, 7, 7, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w64, None, 2, 3).backward(gy.double())
    assert rel_l2(out[16], w64.grad) < 5e-6
    assert rel_l2(out[16], out[1]) < 5e-6
