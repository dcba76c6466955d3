"""Token assembly kernels (csrc/tokens.hip) vs PyTorch on the same inputs.

* fusion tokens (reference model/feature_fusion.py:41-46): drop(cat([bev^T, motion^T
  expanded]) + pos_embed) and its gradients (bev, motion, pos_embed).
* decoder tokens (reference model/control_predict.py:53-54): drop(embedding(tgt) + pos_embed)
  and its gradients (embedding table, pos_embed).
p = 0 (eval / deterministic train): bit-equal to PyTorch's forward (one fp32 add per element);
gradients within 1e-6 (only the order of the sums over the batch / token occurrences
differs).  p > 0: the forward's kept set is exactly the elements the backward passes, with
the 1 / (1 - p) scale, and the kept fraction is ~1 - p; results are deterministic."""
import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _fusion_inputs(B=8, C=256, S=256, E=258, seed=0):
    g = torch.Generator().manual_seed(seed)
    bev = torch.randn(B, C, S, generator=g).to(DEV).requires_grad_()
    motion = torch.randn(B, 1, S, generator=g).to(DEV).requires_grad_()
    pos = (torch.randn(1, S, E, generator=g) * 0.02).to(DEV).requires_grad_()
    return bev, motion, pos


def _fusion_ref(bev, motion, pos):
    E, C = pos.shape[-1], bev.shape[1]
    m = motion.transpose(1, 2).expand(-1, -1, E - C)
    return torch.cat([bev.transpose(1, 2), m], dim=2) + pos


@pytest.mark.parametrize("shape", [(8, 256, 256, 258), (2, 64, 40, 66), (1, 30, 33, 31)])
def test_fusion_tokens_match_torch(shape):
    from e2ep_amd import nn_ops
    B, C, S, E = shape
    bev, motion, pos = _fusion_inputs(B, C, S, E)
    out = nn_ops.fusion_tokens(bev, motion, pos, 0.0)
    ref = _fusion_ref(bev, motion, pos)
    assert torch.equal(out, ref)
    g = torch.randn_like(ref)
    got = torch.autograd.grad(out, (bev, motion, pos), g)
    want = torch.autograd.grad(ref, (bev, motion, pos), g)
    for a, b in zip(got, want):
        assert rel_l2(a, b.double()) < 1e-6


def test_fusion_tokens_dropout_mask_consistent():
    from e2ep_amd import nn_ops
    bev, motion, pos = _fusion_inputs()
    seed = torch.tensor([1234], dtype=torch.int32, device=DEV)
    p = 0.3
    out = nn_ops.fusion_tokens(bev, motion, pos, p, seed)
    full = _fusion_ref(bev, motion, pos).detach()
    kept = out != 0
    assert abs(float(kept.float().mean()) - (1 - p)) < 0.01
    assert torch.allclose(out[kept], full[kept] / (1 - p), rtol=1e-6, atol=0)
    g = torch.ones_like(out)
    dbev, dmotion, dpos = torch.autograd.grad(out, (bev, motion, pos), g)
    scale = kept.float() / (1 - p)  # the backward passes exactly the kept elements
    assert torch.allclose(dbev, scale[:, :, :256].transpose(1, 2), rtol=1e-6)
    assert torch.allclose(dmotion, scale[:, :, 256:].sum(2).unsqueeze(1), rtol=1e-6)
    assert torch.allclose(dpos, scale.sum(0, keepdim=True), rtol=1e-6)
    again = nn_ops.fusion_tokens(bev, motion, pos, p, seed)
    assert torch.equal(out, again)


def _embed_inputs(B=8, T=14, V=204, E=258, seed=0):
    g = torch.Generator().manual_seed(seed)
    gt = torch.randint(0, V, (B, T + 1), generator=g).to(DEV)
    gt[:, 0] = 201
    gt[:, 7] = 203  # PAD rows occur more than once
    table = torch.randn(V, E, generator=g).to(DEV).requires_grad_()
    pos = (torch.randn(1, T, E, generator=g) * 0.02).to(DEV).requires_grad_()
    return gt, table, pos


def test_embed_tokens_match_torch():
    from e2ep_amd import nn_ops
    gt, table, pos = _embed_inputs()
    tgt = gt[:, :-1]  # a strided slice, as the decoder passes it
    out = nn_ops.embed_tokens(tgt, table, pos, 0.0)
    ref = torch.nn.functional.embedding(tgt, table) + pos
    assert torch.equal(out, ref)
    g = torch.randn_like(ref)
    got = torch.autograd.grad(out, (table, pos), g)
    want = torch.autograd.grad(ref, (table, pos), g)
    for a, b in zip(got, want):
        assert rel_l2(a, b.double()) < 1e-6


def test_embed_tokens_dropout_mask_consistent():
    from e2ep_amd import nn_ops
    gt, table, pos = _embed_inputs(B=4, T=14)
    tgt = gt[:, :-1]
    seed = torch.tensor([77], dtype=torch.int32, device=DEV)
    p = 0.5
    out = nn_ops.embed_tokens(tgt, table, pos, p, seed)
    full = (torch.nn.functional.embedding(tgt, table) + pos).detach()
    kept = out != 0
    assert abs(float(kept.float().mean()) - (1 - p)) < 0.03
    assert torch.allclose(out[kept], full[kept] / (1 - p), rtol=1e-6, atol=0)
    dtable, dpos = torch.autograd.grad(out, (table, pos), torch.ones_like(out))
    scale = kept.float() / (1 - p)
    want = torch.zeros_like(dtable).index_add_(0, tgt.reshape(-1), scale.reshape(-1, scale.shape[-1]))
    assert torch.allclose(dtable, want, rtol=1e-6)
    assert torch.allclose(dpos, scale.sum(0, keepdim=True), rtol=1e-6)


def test_embed_tokens_out_of_range_raises_like_embedding():
    """nn.Embedding raises on an id outside [0, V); so does embed_tokens (the kernels' clamp is a
    memory-safety backstop only), for a negative id and for id == V."""
    from e2ep_amd import nn_ops
    table = torch.randn(10, 16, device=DEV)
    pos = torch.randn(1, 3, 16, device=DEV)
    for bad in (-1, 10):
        tok = torch.tensor([[1, bad, 2]], dtype=torch.int64, device=DEV)
        with pytest.raises(IndexError):
            nn_ops.embed_tokens(tok, table, pos)
        with pytest.raises(IndexError):
            torch.nn.functional.embedding(tok.cpu(), table.cpu())


@pytest.mark.parametrize("B,V", [(1, 204), (8, 204), (3, 1000), (2, 7)])
def test_token_argmax_append_matches_softmax_argmax(B, V):
    """e2ep_token_argmax_append (the AR loop's softmax + argmax + cat, reference
    model/control_predict.py:72-75, model/parking_model.py:75-77) writes
    torch.softmax(row).argmax() into column `pos` of the token buffer and nothing else;
    planted exact ties pick the first index, as torch.argmax; e2ep_tokens_init pads with PAD."""
    from e2ep_amd import _lib
    g = torch.Generator().manual_seed(B * V)
    T, L, pad = 14, 2, V - 1
    logits = torch.randn(B, T, V, generator=g) * 3
    logits[:, L - 1, V // 3] = logits[:, L - 1, 2 * V // 3] = logits[:, L - 1].max(-1).values + 1.0
    logits = logits.to(DEV)
    prefix = torch.randint(0, V, (B, 4), generator=g).to(DEV)
    seq = torch.full((B, T), -5, dtype=torch.long, device=DEV)
    s = _lib.stream()
    _lib.call("e2ep_tokens_init", _lib.ptr(prefix), prefix.stride(0), B, L, _lib.ptr(seq), T, pad, s)
    want = seq.clone()
    assert torch.equal(want[:, :L], prefix[:, :L]) and bool((want[:, L:] == pad).all())
    for pos in (L, L + 1):
        row = logits[:, pos - 1, :]
        _lib.call("e2ep_token_argmax_append", _lib.ptr(row), row.stride(0), B, V, _lib.ptr(seq),
                  T, pos, s)
        want[:, pos] = torch.softmax(row, dim=-1).argmax(dim=-1)
    assert torch.equal(seq, want)
    assert bool((seq[:, L] == V // 3).all())  # the first of the two tied maxima
