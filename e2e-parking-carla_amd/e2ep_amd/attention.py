"""torch.nn.MultiheadAttention forward (need_weights=False) on the fused e2ep attention core.

The reference's transformer layers call `self_attn(x, x, x, ...)` / `multihead_attn(x, mem,
mem)` (torch TransformerEncoderLayer / TransformerDecoderLayer, model/feature_fusion.py:13-14,
model/control_predict.py:19-20).  Here the in-projection stays one hipBLASLt GEMM (packed
Q|K|V for self-attention, Q and K|V for cross-attention), the attention core runs as
e2ep_attn_fwd / e2ep_attn_bwd reading Q/K/V in place from that output (no head split
copies, scores never written), and the out-projection is the module's own linear.

`mha(mod, ...)` falls back to calling the module itself whenever the fused path would not be
the same computation or would bypass something a caller installed: forward hooks or an
instance-patched forward (the closed-loop agent's attention capture,
agent/parking_agent.py:71-80,266-268), a float attn_mask not declared causal, bias_k /
add_zero_attn, separate projection weights, or shapes outside the kernel's range.
"""
import math
import os

import torch

from . import _lib, conv, nn_ops, rng, timing

# E2EP_ATTN_SPLIT=1: D first, then dq on the current stream and dk/dv on the side stream.  Off
# by default: the C2 step measured 0.18 ms slower with it (25.58 vs 25.40 ms/step,
# profiles/r02/session6/attn_split_ab.txt) — the two passes contend for the same CUs and the
# extra D launch is on the critical path.
_SPLIT_BWD = os.environ.get("E2EP_ATTN_SPLIT", "0") == "1"

MAX_SEQ = 256
MAX_HEAD_DIM = 64


class _Attn(torch.autograd.Function):
    """O = dropout_p(softmax(scale Q K^T + mask)) V on (S, B, E)-strided Q/K/V, or (B, S, E)
    with batch_first (the kernels take sequence / batch strides; the dropout counters index
    the logical (b, h, i, j), so both layouts draw the same masks).

    `qb` holds Q at column offset 0 (row stride qb.shape[-1]); `kvb` holds K at column offset
    `k_off` and V at `k_off + E`.  When kvb is None, K/V live in qb itself (packed QKV)."""

    @staticmethod
    def forward(ctx, qb, kvb, H, causal, key_pad, p, seed, batch_first=False):
        packed = kvb is None
        kvt = qb if packed else kvb
        if batch_first:
            B, Sq, Wq = qb.shape
            _, Sk, Wkv = kvt.shape
        else:
            Sq, B, Wq = qb.shape
            Sk, _, Wkv = kvt.shape
        E = Wq // 3 if packed else Wq
        dh = E // H
        k_off = E if packed else 0
        oshape = (B, Sq, E) if batch_first else (Sq, B, E)
        o = torch.empty(oshape, dtype=qb.dtype, device=qb.device)
        lse = torch.empty(B * H, Sq, dtype=torch.float32, device=qb.device)
        kptr = kvt.data_ptr() + 4 * k_off
        vptr = kptr + 4 * E
        if batch_first:  # (sequence, batch) strides
            dims = (B, H, Sq, Sk, dh, Wq, Sq * Wq, Wkv, Sk * Wkv, E, Sq * E)
        else:
            dims = (B, H, Sq, Sk, dh, B * Wq, Wq, B * Wkv, Wkv, B * E, E)
        with timing.region("attn_fwd"):
            _lib.call("e2ep_attn_fwd", _lib.ptr(qb), kptr, vptr, *dims, 1.0 / math.sqrt(dh),
                      int(causal), _lib.ptr(key_pad), float(p), _lib.ptr(seed), _lib.ptr(o),
                      _lib.ptr(lse), _lib.stream())
        ctx.save_for_backward(qb, kvb, o, lse, key_pad, seed)
        ctx.cfg = (packed, dims, E, k_off, causal, float(p))
        return o

    @staticmethod
    def backward(ctx, do):
        qb, kvb, o, lse, key_pad, seed = ctx.saved_tensors
        packed, dims, E, k_off, causal, p = ctx.cfg
        B, H, Sq = dims[0], dims[1], dims[2]
        kvt = qb if packed else kvb
        do = do.contiguous()
        dqb = torch.empty_like(qb)
        dkvb = None if packed else torch.empty_like(kvb)
        dkvt = dqb if packed else dkvb
        kptr = kvt.data_ptr() + 4 * k_off
        dkptr = dkvt.data_ptr() + 4 * k_off
        ws = torch.empty(_lib.call_raw("e2ep_attn_bwd_workspace", B, H, Sq) // 4,
                         dtype=torch.float32, device=qb.device)
        args = (_lib.ptr(qb), kptr, kptr + 4 * E, _lib.ptr(o), _lib.ptr(do), _lib.ptr(lse), *dims,
                1.0 / math.sqrt(dims[4]), int(causal), _lib.ptr(key_pad), p, _lib.ptr(seed),
                _lib.ptr(dqb), dkptr, dkptr + 4 * E, _lib.ptr(ws))
        with timing.region("attn_bwd"):
            if not (conv.wgrad_overlap() and _SPLIT_BWD):  # serial (A/B, per-kernel timing)
                _lib.call("e2ep_attn_bwd_part", *args, 0, _lib.stream())
            else:
                # D first, then dq here and dk/dv on the side stream concurrently (conv._Fork:
                # every buffer is allocated above, on the current stream)
                _lib.call("e2ep_attn_bwd_part", *args, 1, _lib.stream())
                # dk / dv: ~4 dh-long fma chains per (query, key) pair and head, vector rate
                B_, H_, Sq_, Sk_, dh_ = dims[:5]
                fork = conv._Fork(qb.device, work_us=conv.est_us(
                    8.0 * B_ * H_ * Sq_ * Sk_ * dh_ * 4))
                with fork:
                    _lib.call("e2ep_attn_bwd_part", *args, 3, _lib.stream())
                _lib.call("e2ep_attn_bwd_part", *args, 2, _lib.stream())
                fork.join()
        return dqb, dkvb, None, None, None, None, None, None


def attention(qb, kvb, H, causal=False, key_pad=None, p=0.0, seed=None, batch_first=False):
    """Functional entry: see _Attn.  key_pad: bool (B, Sk) or None; seed: int32 (1,) device
    tensor, drawn here when p > 0 and none is given; batch_first: (B, S, .) operands and
    output instead of (S, B, .)."""
    if p > 0.0 and seed is None:
        seed = rng.seed(qb.device)
    qb = qb.contiguous()
    kvb = None if kvb is None else kvb.contiguous()
    if key_pad is not None:
        key_pad = key_pad.contiguous()
        if key_pad.dtype != torch.bool:
            raise TypeError("key_pad must be a bool mask (True = ignore key)")
    return _Attn.apply(qb, kvb, H, bool(causal), key_pad, float(p), seed, bool(batch_first))


def _fusable(mod, query, key, attn_mask, key_padding_mask, is_causal, batch_first=False):
    if key_padding_mask is not None and key_padding_mask.dtype != torch.bool:
        return False
    if mod._forward_hooks or mod._forward_pre_hooks or "forward" in mod.__dict__:
        return False
    if not mod._qkv_same_embed_dim or mod.batch_first or mod.bias_k is not None or mod.add_zero_attn:
        return False
    if attn_mask is not None and not is_causal:
        return False
    if not query.is_cuda or query.dtype != torch.float32 or query.dim() != 3:
        return False
    E, H = mod.embed_dim, mod.num_heads
    sd = 1 if batch_first else 0  # sequence dim
    return (E // H <= MAX_HEAD_DIM and query.shape[sd] <= MAX_SEQ and key.shape[sd] <= MAX_SEQ)


def mha(mod, query, key, value, attn_mask=None, key_padding_mask=None, is_causal=False,
        skip=False, kv_skip=False, batch_first=False):
    """mod(query, key, value, attn_mask=..., key_padding_mask=..., need_weights=False)[0] for a
    seq-first nn.MultiheadAttention, on the fused core when possible.  `is_causal` asserts
    that attn_mask is the causal (-inf above the diagonal) mask, as torch's is_causal hint.
    skip=True returns (out, query_skip): the layer's residual reads query_skip, whose gradient
    the query projection's input-gradient GEMM accumulates (nn_ops.linear).  kv_skip=True
    (cross attention, key is value) appends key_skip, to be used as the key/value input of the
    next consumer (the next decoder layer's memory).  batch_first: (B, S, E) query / key /
    value and output (the module itself stays seq-first: its fallback call gets transposes)."""
    def ret(out, qs, ks):
        r = (out,) + ((qs,) if skip else ()) + ((ks,) if kv_skip else ())
        return r if len(r) > 1 else out

    def t(z):
        return z.transpose(0, 1) if batch_first else z

    if not _fusable(mod, query, key, attn_mask, key_padding_mask, is_causal, batch_first):
        out = mod(t(query), t(key), t(value), attn_mask=attn_mask,
                  key_padding_mask=key_padding_mask, need_weights=False,
                  is_causal=bool(is_causal) and attn_mask is not None)[0]
        return ret(t(out), query, key)
    E, H = mod.embed_dim, mod.num_heads
    W, bias = mod.in_proj_weight, mod.in_proj_bias
    p = mod.dropout if mod.training else 0.0
    if query is key and key is value:
        qkv, qs = nn_ops.linear(query, W, bias, skip=True)
        ks = qs  # self attention: one input (kv_skip is for cross attention)
        o = attention(qkv, None, H, is_causal, key_padding_mask, p, batch_first=batch_first)
    else:
        if key is not value:
            out = mod(t(query), t(key), t(value), attn_mask=attn_mask,
                      key_padding_mask=key_padding_mask, need_weights=False)[0]
            return ret(t(out), query, key)
        # one Function over the whole in_proj_weight: its backward writes the q and kv row
        # blocks of dW / db in place (a weight split would concatenate them: 2 cat launches)
        q, kv, qs, ks = nn_ops.in_proj_qkv(query, key, W, bias, E)
        o = attention(q, kv, H, is_causal, key_padding_mask, p, batch_first=batch_first)
    out = nn_ops.linear(o, mod.out_proj.weight, mod.out_proj.bias)
    return ret(out, qs, ks)
