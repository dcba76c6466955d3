"""Conv GEMM operand precision (e2ep_conv_precision): "fp32" (default, exact-f32 MFMA),
"bf16" (BASELINE C3: bf16 forward, fp32 gradients) and "fp16" (C5 inference).

Low precision applies to the conv GEMMs: their operands are rounded to bf16 / fp16 as they
enter the matrix cores, products and sums stay fp32, every tensor stays fp32 in HBM.  "bf16"
(training, AMP-style) covers the forward, data-gradient and weight-gradient GEMMs — the weight
gradients are accumulated and stored in fp32; "fp16" (inference) covers the forward and
data-gradient GEMMs.  BatchNorm, depthwise convs, attention, the transformer linears, the
losses, the optimizer and the gradient all-reduce stay fp32.  The setting is process-wide
(one library state); `use` restores the previous mode."""
from contextlib import contextmanager

from . import _lib

MODES = {"fp32": 0, "bf16": 1, "fp16": 2}
_NAMES = {v: k for k, v in MODES.items()}


def set(mode):  # noqa: A001 - mirrors torch.set_* naming
    """Select the mode; returns the previous one."""
    if mode not in MODES:
        raise ValueError(f"precision must be one of {sorted(MODES)}, got {mode!r}")
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
