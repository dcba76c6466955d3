"""Transformer encoder/decoder stacks of the fusion and control-decoder modules.

d_model 258, 6 heads x 43, FFN 2048, post-norm, ReLU (reference model/feature_fusion.py:13-14,
model/control_predict.py:19-20).  The layers stay torch.nn Transformer*Layer modules (state-dict
keys and the agent's self_attn hook, agent/parking_agent.py:71-80); their forward is restated
here with the same math and the same submodules, except that each "x + dropout(sublayer(x))
-> LayerNorm" runs as one e2ep kernel (nn_ops.add_drop_layer_norm) instead of PyTorch's
dropout + add + layer_norm (+ its slow gamma/beta backward).  The attention core (QK^T, mask,
softmax, dropout, PV and their backward) runs as e2ep kernels through attention.mha, which
keeps the modules' own in/out projections (hipBLASLt GEMMs) and falls back to the module when
a hook is installed (the agent's attention capture)."""

import torch
import torch.nn.functional as F

from . import attention, nn_ops


def _p(drop, training):
    return drop.p if training else 0.0


def _ff(layer, x):
    """(linear2(dropout(relu(linear1(x)))), x_skip) — x_skip carries the residual (see
    nn_ops.linear skip)."""
    h, xs = nn_ops.linear(x, layer.linear1.weight, layer.linear1.bias, skip=True)
    if layer.activation is F.relu and h.is_cuda and h.dtype == torch.float32 and h.numel() % 4 == 0:
        h = nn_ops.relu_dropout(h, _p(layer.dropout, layer.training))  # one launch each way
    else:
        h = layer.dropout(layer.activation(h))
    return nn_ops.linear(h, layer.linear2.weight, layer.linear2.bias), xs


def encoder_layer(layer, x, mask=None, key_padding_mask=None, batch_first=False):
    """torch.nn.TransformerEncoderLayer.forward (norm_first=False), seq-first x (S, B, E), or
    (B, S, E) with batch_first (the same math: the linears and LayerNorms are row-wise)."""
    assert not layer.norm_first
    sa, x = attention.mha(layer.self_attn, x, x, x, attn_mask=mask,
                          key_padding_mask=key_padding_mask, skip=True, batch_first=batch_first)
    x = nn_ops.add_drop_layer_norm(x, sa, layer.norm1, _p(layer.dropout1, layer.training))
    ff, x = _ff(layer, x)
    return nn_ops.add_drop_layer_norm(x, ff, layer.norm2, _p(layer.dropout2, layer.training))


def decoder_layer(layer, x, memory, tgt_mask=None, tgt_key_padding_mask=None, tgt_is_causal=False,
                  batch_first=False):
    """torch.nn.TransformerDecoderLayer.forward (norm_first=False), seq-first.  Returns
    (out, memory_skip): the next layer reads memory_skip, so the memory's gradients from all
    layers are summed in the in-projection GEMM epilogues (no autograd adds)."""
    assert not layer.norm_first
    sa, x = attention.mha(layer.self_attn, x, x, x, attn_mask=tgt_mask,
                          key_padding_mask=tgt_key_padding_mask, is_causal=bool(tgt_is_causal),
                          skip=True, batch_first=batch_first)
    x = nn_ops.add_drop_layer_norm(x, sa, layer.norm1, _p(layer.dropout1, layer.training))
    ca, x, memory = attention.mha(layer.multihead_attn, x, memory, memory, skip=True, kv_skip=True,
                                  batch_first=batch_first)
    x = nn_ops.add_drop_layer_norm(x, ca, layer.norm2, _p(layer.dropout2, layer.training))
    ff, x = _ff(layer, x)
    return nn_ops.add_drop_layer_norm(x, ff, layer.norm3, _p(layer.dropout3, layer.training)), memory


def encoder(stack, tokens):
    """tokens (B, S, E) batch-first -> (B, S, E).  The reference runs the stack seq-first; here
    the layers run batch-first on the same rows (no transposed copies of the activations or
    their gradients: the attention kernels take (sequence, batch) strides)."""
    x = tokens
    for layer in stack.layers:
        x = encoder_layer(layer, x, batch_first=True)
    if stack.norm is not None:
        x = stack.norm(x)
    return x


def decoder(stack, tgt, memory, tgt_mask, tgt_key_padding_mask, tgt_is_causal=None):
    """tgt (B, T, E), memory (B, S, E) batch-first -> (B, T, E) (see encoder)."""
    x, mem = tgt, memory
    for layer in stack.layers:
        x, mem = decoder_layer(layer, x, mem, tgt_mask, tgt_key_padding_mask, tgt_is_causal,
                               batch_first=True)
    if stack.norm is not None:
        x = stack.norm(x)
    return x
