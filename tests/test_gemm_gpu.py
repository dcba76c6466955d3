"""e2ep_gemm (csrc/gemm.hip) and the nn.Linear built on it (e2ep_amd.nn_ops.linear) vs fp64
PyTorch: every operand layout the linear uses (forward (A k-contig, B k-contig), input
gradient (A k-contig, B n-contig), weight gradient (A m-contig, B n-contig)) plus the fourth,
at the transformer shapes of the C2 step (2048 encoder rows, 112 decoder rows, d = 258, FFN
2048), the C5 decoder's 14 rows (the skinny wave-per-column kernel for M <= 16) and ragged edges (M, N, K not multiples of the tiles; K = 1..3).
Tolerance: rel-L2 <= 2e-6 against fp64 (fp32 MFMA products are exact, accumulation is
fp32 over at most 2048 terms); split-K results bitwise identical across launches."""
import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [(2048, 774, 258), (2048, 258, 2048), (258, 2048, 2048), (774, 258, 2048),
          (112, 516, 258), (112, 204, 258), (8, 64, 3), (8, 256, 128), (1, 1, 1), (65, 130, 17),
          (3, 5, 700), (200, 3, 64), (14, 2048, 258), (16, 258, 2048), (14, 205, 258)]


def _operands(M, N, K, ak, bk, g):
    A = torch.randn(M, K, generator=g) if ak else torch.randn(K, M, generator=g)
    B = torch.randn(N, K, generator=g) if bk else torch.randn(K, N, generator=g)
    Am = A if ak else A.t()
    Bm = B.t() if bk else B
    return A, B, Am.double() @ Bm.double()


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_layouts_vs_fp64(M, N, K, ak, bk):
    from e2ep_amd import nn_ops
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + 11 * ak + 5 * bk)
    A, B, ref = _operands(M, N, K, ak, bk, g)
    out = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K)
    assert rel_l2(out, ref) < 2e-6
    again = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K)
    assert torch.equal(out, again)


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_every_tile_and_split(tile, ak, bk):
    """Each block tile (e2ep_gemm_force) with and without a K split, ragged M / N / K, plus
    the bias + residual + ReLU epilogue (written directly, or by the split reduction)."""
    from e2ep_amd import _lib, nn_ops
    M, N, K = 197, 301, 333
    g = torch.Generator().manual_seed(tile * 10 + 2 * ak + bk)
    A, B, ref = _operands(M, N, K, ak, bk, g)
    bias, cadd = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    want = (ref + bias.double() + cadd.double()).clamp_min(0)
    try:
        for splits in (1, 3):
            _lib.call("e2ep_gemm_force", tile, splits, 0)
            out = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K)
            assert rel_l2(out, ref) < 2e-6, (tile, splits)
            out = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K, bias=bias.to(DEV),
                              cadd=cadd.to(DEV), relu=True)
            assert rel_l2(out, want) < 2e-6, (tile, splits)
    finally:
        _lib.call("e2ep_gemm_force", 0, 0, 0)


@pytest.mark.parametrize("M,N,K", [(2048, 258, 258), (112, 204, 258), (37, 70, 2048),
                                   (14, 2048, 258), (15, 258, 2048), (7, 33, 17)])
def test_gemm_epilogue_bias_add_relu(M, N, K):
    from e2ep_amd import nn_ops
    g = torch.Generator().manual_seed(M + N + K)
    A, B, ref = _operands(M, N, K, True, True, g)
    bias, cadd = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    out = nn_ops.gemm(A.to(DEV), True, B.to(DEV), True, M, N, K, bias=bias.to(DEV),
                      cadd=cadd.to(DEV), relu=True)
    want = (ref + bias.double() + cadd.double()).clamp_min(0)
    assert rel_l2(out, want) < 2e-6
    assert float(out.min()) >= 0.0


def test_gemm_strided_operands():
    """Row slices of a bigger matrix (in_proj_weight[E:] for the cross-attention K/V)."""
    from e2ep_amd import nn_ops
    g = torch.Generator().manual_seed(3)
    W = torch.randn(774, 258, generator=g).to(DEV)
    x = torch.randn(2048, 300, generator=g).to(DEV)[:, :258]     # lda = 300
    out = nn_ops.gemm(x, True, W[258:], True, 2048, 516, 258)
    ref = x.double() @ W[258:].double().t()
    assert rel_l2(out, ref) < 2e-6


@pytest.mark.parametrize("shape,relu,skip", [((8, 256, 258), False, True), ((8, 14, 258), False, False),
                                             ((8, 1, 3), True, False)])
def test_linear_autograd_vs_fp64(shape, relu, skip):
    from e2ep_amd import nn_ops
    g = torch.Generator().manual_seed(len(shape) + shape[-1])
    K = shape[-1]
    N = 204 if K == 258 and not skip else 64 if K == 3 else 774
    x = torch.randn(*shape, generator=g)
    W = torch.randn(N, K, generator=g) * 0.1
    b = torch.randn(N, generator=g)
    gy = torch.randn(*shape[:-1], N, generator=g)
    gs = torch.randn(*shape, generator=g)
    xr, Wr, br = (t.double().requires_grad_() for t in (x, W, b))
    yr = torch.nn.functional.linear(xr, Wr, br)
    if relu:
        yr = yr.clamp_min(0)
    loss_r = (yr * gy.double()).sum() + ((xr * gs.double()).sum() if skip else 0)
    loss_r.backward()
    xd, Wd, bd = (t.to(DEV).requires_grad_() for t in (x, W, b))
    out = nn_ops.linear(xd, Wd, bd, skip=skip, relu=relu)
    if skip:
        y, xs = out
        loss = (y * gy.to(DEV)).sum() + (xs * gs.to(DEV)).sum()
    else:
        y = out
        loss = (y * gy.to(DEV)).sum()
    loss.backward()
    assert rel_l2(y, yr) < 2e-6
    assert rel_l2(xd.grad, xr.grad) < 2e-6
    assert rel_l2(Wd.grad, Wr.grad) < 2e-6
    assert rel_l2(bd.grad, br.grad) < 2e-6


def test_gemm_rejects_bad_shapes():
    from e2ep_amd import _lib, nn_ops
    A = torch.randn(4, 5, device=DEV)
    with pytest.raises(_lib.E2EPError):
        nn_ops.gemm(A, True, torch.randn(3, 6, device=DEV), True, 4, 3, 5)
    with pytest.raises(_lib.E2EPError):
        nn_ops.gemm(A.t(), True, torch.randn(3, 5, device=DEV), True, 5, 3, 4)
    with pytest.raises(_lib.E2EPError):
        nn_ops.linear(torch.randn(2, 5), torch.randn(3, 5), None)


def _rowsum_gemm(g2, x2):
    """dW = g2^T x2 and db = g2.sum(0) through the one-launch e2ep_gemm_rowsum."""
    from e2ep_amd import _lib
    rows, N = g2.shape
    K = x2.shape[1]
    dw = torch.empty(N, K, dtype=torch.float32, device=DEV)
    db = torch.empty(N, dtype=torch.float32, device=DEV)
    nb = _lib.load().e2ep_gemm_rowsum_workspace(N, K, rows)
    ws = torch.empty(max(1, nb // 4), dtype=torch.float32, device=DEV)
    _lib.call("e2ep_gemm_rowsum", _lib.ptr(g2), g2.stride(0), _lib.ptr(x2), x2.stride(0),
              _lib.ptr(dw), K, _lib.ptr(db), N, K, rows, _lib.ptr(ws), _lib.nbytes(ws), _lib.stream())
    return dw, db


@pytest.mark.parametrize("rows,N,K", [(2048, 774, 258), (2048, 258, 2048), (2048, 2048, 258),
                                      (112, 258, 258), (112, 204, 258), (24, 64, 15),
                                      (37, 70, 100), (5, 3, 32), (300, 33, 64)])
def test_gemm_rowsum_weight_and_bias_gradient(rows, N, K):
    """Linear backward's dW = dY^T X with db = dY.sum(0) taken by the same launch (a ones column
    appended to X): both vs fp64, for widths where the ones column lands in a partial tile
    (K % 32 != 0) and where it needs a tile of its own (K % 64 == 0), with and without K split."""
    g = torch.Generator().manual_seed(rows + 3 * N + K)
    g2, x2 = torch.randn(rows, N, generator=g), torch.randn(rows, K, generator=g)
    dw, db = _rowsum_gemm(g2.to(DEV), x2.to(DEV))
    assert rel_l2(dw, g2.double().t() @ x2.double()) < 2e-6
    assert rel_l2(db, g2.double().sum(0)) < 2e-6
    dw2, db2 = _rowsum_gemm(g2.to(DEV), x2.to(DEV))
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
def test_gemm_rowsum_every_tile_and_split(tile):
    from e2ep_amd import _lib
    rows, N, K = 333, 197, 256
    g = torch.Generator().manual_seed(tile)
    g2, x2 = torch.randn(rows, N, generator=g), torch.randn(rows, K, generator=g)
    try:
        for splits in (1, 3):
            _lib.call("e2ep_gemm_force", tile, splits, 0)
            dw, db = _rowsum_gemm(g2.to(DEV), x2.to(DEV))
            assert rel_l2(dw, g2.double().t() @ x2.double()) < 2e-6, (tile, splits)
            assert rel_l2(db, g2.double().sum(0)) < 2e-6, (tile, splits)
    finally:
        _lib.call("e2ep_gemm_force", 0, 0, 0)


def test_linear_bias_gradient_from_rowsum_launch():
    """nn_ops.linear backward: weight and bias gradients (one e2ep_gemm_rowsum launch) and the
    bias-only case (e2ep_col_sum) against fp64 autograd."""
    from e2ep_amd import nn_ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 50, 258, generator=g)
    w = torch.randn(774, 258, generator=g) / 16
    b = torch.randn(774, generator=g)
    dy = torch.randn(4, 50, 774, generator=g)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    nn_ops.linear(xd, wd, bd).backward(dy.to(DEV))
    x64, w64, b64 = (t.double().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.linear(x64, w64, b64).backward(dy.double())
    assert rel_l2(wd.grad, w64.grad) < 2e-6
    assert rel_l2(bd.grad, b64.grad) < 2e-6
    assert rel_l2(xd.grad, x64.grad) < 2e-6
    wf = w.to(DEV)  # frozen weight: bias gradient alone
    bd.grad = None
    nn_ops.linear(xd.detach(), wf, bd).backward(dy.to(DEV))
    assert rel_l2(bd.grad, b64.grad) < 2e-6


@pytest.mark.parametrize("M,N,K", [(2048, 774, 258), (258, 2048, 2048), (112, 516, 258),
                                   (65, 130, 17), (2048, 258, 2048)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False)])
def test_gemm_bf16_operands_vs_rounded_fp64(M, N, K, ak, bk):
    """C3 (e2ep_gemm_precision 1): bf16 operands, fp32 products and sums — against fp64 of the
    bf16-rounded operands (rel-L2 2e-6: only the fp32 accumulation differs), and the rounding
    really happens (the unrounded fp64 product is ~1e-3 away)."""
    from e2ep_amd import nn_ops, precision
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + ak + 2 * bk)
    A, B, ref = _operands(M, N, K, ak, bk, g)
    Ar, Br = A.bfloat16().double(), B.bfloat16().double()
    want = (Ar if ak else Ar.t()) @ (Br.t() if bk else Br)
    with precision.use("bf16"):
        out = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K)
        again = nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K)
    assert rel_l2(out, want) < 2e-6
    assert torch.equal(out, again)
    if K >= 64:
        assert rel_l2(out, ref) > 1e-4
    assert rel_l2(nn_ops.gemm(A.to(DEV), ak, B.to(DEV), bk, M, N, K), ref) < 2e-6  # fp32 again


def test_short_workspace_is_rejected():
    """Every workspace-taking entry point gets the workspace size and refuses (E2EP_EINVAL,
    nothing launched) a buffer smaller than its launch plan needs: a K-split
    GEMM and a conv weight gradient with their workspaces one float short."""
    from e2ep_amd import _lib
    M, N, K = 197, 301, 777
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV)
    C = torch.empty(M, N, device=DEV)
    try:
        _lib.call("e2ep_gemm_force", 1, 3, 0)
        need = _lib.load().e2ep_gemm_workspace(M, N, K)
        assert need > 0
        ws = torch.empty(need // 4, device=DEV)
        args = lambda w, nb: (_lib.ptr(A), K, 1, _lib.ptr(B), K, 1, None, None, 0, _lib.ptr(C), N,  # noqa: E731
                              M, N, K, 0, _lib.ptr(w), nb, _lib.stream())
        _lib.call("e2ep_gemm", *args(ws, _lib.nbytes(ws)))
        with pytest.raises(_lib.E2EPError, match="workspace"):
            _lib.call("e2ep_gemm", *args(ws, _lib.nbytes(ws) - 4))
    finally:
        _lib.call("e2ep_gemm_force", 0, 0, 0)
    d = _lib.dims((2, 64, 16, 16, 64, 3, 3, 16, 16, 1, 1, 1, 1, 1, 1))
    splits = _lib.load().e2ep_conv_wgrad_splits(d)
    nb = _lib.load().e2ep_conv_wgrad_workspace(d, splits)
    gy, x = torch.randn(2, 64, 16, 16, device=DEV), torch.randn(2, 64, 16, 16, device=DEV)
    dw, ws = torch.empty(64, 64, 3, 3, device=DEV), torch.empty(nb // 4, device=DEV)
    with pytest.raises(_lib.E2EPError, match="workspace"):
        _lib.call("e2ep_conv_wgrad", _lib.ptr(gy), _lib.ptr(x), d, splits, _lib.ptr(ws), nb - 4,
                  _lib.ptr(dw), 0, _lib.stream(), 0)
    torch.cuda.synchronize()


# (rows M, out N, in K): the control decoder (B = 8: 112 rows; 14 tokens x 8), the fusion
# encoder (2048 rows), the FFN, odd shapes that split K and pad every tile edge
PAIR_SHAPES = [(112, 258, 258), (112, 774, 258), (112, 2048, 258), (112, 258, 2048),
               (2048, 258, 258), (2048, 2048, 258), (97, 130, 333), (33, 64, 1500)]


@pytest.mark.parametrize("shape", PAIR_SHAPES, ids=[str(s) for s in PAIR_SHAPES])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_linear_bwd_pair_bitwise_equals_two_launches(shape, skip, prec):
    """e2ep_linear_bwd (dX, dW and db in one k_gemm_pair launch) == e2ep_gemm + e2ep_gemm_rowsum
    launched separately, bit for bit, for fp32 and bf16 operands; and close to fp64."""
    from e2ep_amd import _lib, nn_ops, precision
    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K)
    dy = torch.randn(M, N, generator=g).to(DEV)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    gs = torch.randn(M, K, generator=g).to(DEV) if skip else None
    _linear_pair_case(_lib.load(), dy, x, w, gs, M, N, K, skip, prec)


def _linear_pair_case(lib, dy, x, w, gs, M, N, K, skip, prec):
    from e2ep_amd import _lib, nn_ops, precision
    with precision.use(prec):
        dx = torch.empty(M, K, device=DEV)
        dw = torch.empty(N, K, device=DEV)
        db = torch.empty(N, device=DEV)
        wsx = torch.empty(max(16, lib.e2ep_gemm_workspace(M, K, N)), dtype=torch.uint8, device=DEV)
        wsw = torch.empty(max(16, lib.e2ep_gemm_rowsum_workspace(N, K, M)), dtype=torch.uint8, device=DEV)
        _lib.call("e2ep_linear_bwd", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(gs),
                  K if skip else 0, _lib.ptr(dx), K, _lib.ptr(dw), K, _lib.ptr(db), M, N, K,
                  _lib.ptr(wsx), _lib.nbytes(wsx), _lib.ptr(wsw), _lib.nbytes(wsw), _lib.stream())
        dx2 = nn_ops.gemm(dy, True, w, False, M, K, N, cadd=gs)
        dw2 = torch.empty(N, K, device=DEV)
        db2 = torch.empty(N, device=DEV)
        _lib.call("e2ep_gemm_rowsum", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(dw2), K, _lib.ptr(db2),
                  N, K, M, _lib.ptr(wsw), _lib.nbytes(wsw), _lib.stream())
        torch.cuda.synchronize()
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)
    if prec == "fp32":
        want_dx = dy.double() @ w.double() + (gs.double() if skip else 0)
        assert rel_l2(dx, want_dx) < 2e-6
        assert rel_l2(dw, dy.double().t() @ x.double()) < 2e-6
        assert rel_l2(db, dy.double().sum(0)) < 2e-6


def test_linear_bwd_pair_fallback_with_forced_tiles():
    """With a benchmark-forced tile the pair falls back to two launches on one stream: same
    results."""
    from e2ep_amd import _lib
    M, N, K = 112, 258, 258
    g = torch.Generator().manual_seed(4)
    dy, x = torch.randn(M, N, generator=g).to(DEV), torch.randn(M, K, generator=g).to(DEV)
    w = torch.randn(N, K, generator=g).to(DEV)
    lib = _lib.load()
    outs = []
    for forced in (False, True):
        if forced:
            _lib.call("e2ep_gemm_force", 4, 1, 0)
        try:
            dx, dw, db = torch.empty(M, K, device=DEV), torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
            wsx = torch.empty(max(16, lib.e2ep_gemm_workspace(M, K, N)), dtype=torch.uint8, device=DEV)
            wsw = torch.empty(max(16, lib.e2ep_gemm_rowsum_workspace(N, K, M)), dtype=torch.uint8, device=DEV)
            _lib.call("e2ep_linear_bwd", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(w), K, None, 0,
                      _lib.ptr(dx), K, _lib.ptr(dw), K, _lib.ptr(db), M, N, K, _lib.ptr(wsx),
                      _lib.nbytes(wsx), _lib.ptr(wsw), _lib.nbytes(wsw), _lib.stream())
            outs.append((dx, dw, db))
        finally:
            _lib.call("e2ep_gemm_force", 0, 0, 0)
    for a, b in zip(*outs):
        assert rel_l2(a, b.double()) < 2e-6
