"""GEMM operand precision: "fp32" (default, exact-f32 MFMA), "bf16" (BASELINE C3: bf16
forward, fp32 gradients) and "fp16" (C5 inference).

Low precision rounds the operands of the matrix-core GEMMs to bf16 / fp16 as they enter the
MFMA units; products and sums stay fp32 and every tensor stays fp32 in HBM.  "bf16" (training,
AMP-style) covers the conv GEMMs (forward, data gradient, weight gradient; e2ep_conv_precision)
and the transformer linears (forward, input gradient, weight gradient; e2ep_gemm_precision):
weight gradients are accumulated and stored in fp32.  "fp16" (inference) covers the conv
forward and data-gradient GEMMs; the linears stay fp32 there.  BatchNorm, depthwise convs,
attention (vector-ALU kernels), the losses, the optimizer and the gradient all-reduce stay fp32
in every mode.  The setting is process-wide (one library state); `use` restores the previous
mode."""
from contextlib import contextmanager

from . import _lib

MODES = {"fp32": 0, "bf16": 1, "fp16": 2}
_NAMES = {v: k for k, v in MODES.items()}


def set(mode):  # noqa: A001 - mirrors torch.set_* naming
    """Select the mode; returns the previous one."""
    if mode not in MODES:
        raise ValueError(f"precision must be one of {sorted(MODES)}, got {mode!r}")
    _lib.call_raw("e2ep_gemm_precision", 1 if mode == "bf16" else 0)
    return _NAMES[_lib.call_raw("e2ep_conv_precision", MODES[mode])]


def get():
    return _NAMES[_lib.call_raw("e2ep_conv_precision", -1)]


@contextmanager
def use(mode):
    old = set(mode)
    try:
        yield
    finally:
        set(old)
