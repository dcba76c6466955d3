"""Transformer encoder/decoder stacks of the fusion and control-decoder modules.

d_model 258, 6 heads x 43, FFN 2048, post-norm, ReLU (reference model/feature_fusion.py:13-14,
model/control_predict.py:19-20).  The layers are kept as torch.nn Transformer*Layer modules
(state-dict keys and the agent's self_attn hook, agent/parking_agent.py:71-80); the arithmetic
is routed here so the GEMMs/attention can run on e2ep kernels."""


def encoder(stack, tokens):
    """tokens (B, S, E) batch-first -> (B, S, E); the reference runs the stack seq-first."""
    return stack(tokens.transpose(0, 1)).transpose(0, 1)


def decoder(stack, tgt, memory, tgt_mask, tgt_key_padding_mask, tgt_is_causal=None):
    y = stack(tgt=tgt.transpose(0, 1), memory=memory.transpose(0, 1), tgt_mask=tgt_mask,
              tgt_key_padding_mask=tgt_key_padding_mask, tgt_is_causal=tgt_is_causal)
    return y.transpose(0, 1)
