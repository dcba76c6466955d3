"""Independent model branches on side streams (MI355X: many of the step's launches fill a
fraction of the 256 CUs — 16x16 camera maps, the transformer's token rows — so two
independent chains of them overlap instead of running back to back).

    with branch("cam", device) as br:
        depth = depth_head(deep, skip)          # on a side stream
    feature = feature_head(deep, skip)          # on the current stream, concurrently
    depth = br.join(depth)                      # the current stream waits for the side stream

The branch's ops are ordinary autograd ops recorded on the side stream, so their backward
also runs there (PyTorch's stream semantics for autograd: a node's backward runs on its
forward's stream, synchronised with the streams its incoming gradients come from, and the
engine makes the caller wait for every stream it used before backward() returns), and a
HIP-graph capture of the step records both chains as parallel branches.  Tensors that cross
between the streams are handed to the caching allocator with record_stream, so their memory
is not recycled while the other stream may still use it.

No stream is forked from a branch's stream: the conv / depthwise / linear backward's
weight-gradient fork (conv._Fork) stays on the branch stream there.  With such nested forks a
HIP-graph capture of the train step segfaulted inside hipStreamEndCapture (rounds 2 and 4);
without them the same capture replays correctly (scripts/diag_branch_capture.py, variants
model_cam / model_cam_nofork).

Branches are named so each can be switched off for A/B timing: E2EP_BRANCH_STREAMS is a
comma list of enabled names, "none" for none (default: both; replayed C2 step 22.78 -> 21.73
ms, C3 19.94 -> 18.84 ms, profiles/r05/branch_streams_ab.txt):
  cam    the camera encoder's depth head next to its feature head (model/cam_encoder.py)
  heads  the segmentation head next to the control decoder (model/parking_model.py)
"""
import os

import torch

_ENABLED = set(x for x in os.environ.get("E2EP_BRANCH_STREAMS", "cam,heads").split(",")
               if x and x != "none")
_STREAMS = {}


def enabled(name):
    return name in _ENABLED


def set_enabled(names):
    """Replace the enabled set (returns the previous one)."""
    global _ENABLED
    prev = set(_ENABLED)
    _ENABLED = set(names)
    return prev


def is_branch_stream(stream):
    """True when `stream` is one of the branch side streams."""
    return any(stream == st for st in _STREAMS.values())


def _side(device, name):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, name)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(device=idx)
    return st


class branch:
    """Context manager running its body on a side stream forked from the current stream.
    training=False (an inference forward: predict, validation) keeps the body on the current
    stream: at B = 1 the fork / join costs more than the overlap gains (C5 predict p50 4.41 ms
    with the branches, 4.20 ms without, profiles/r05/c5_ab.txt)."""

    def __init__(self, name, device, inputs=(), training=True):
        self.on = training and enabled(name) and device.type == "cuda"
        self.device, self.name, self.inputs = device, name, inputs
        if self.on:
            self.main = torch.cuda.current_stream(device)
            self.side = _side(device, name)

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            for t in self.inputs:  # produced on the current stream, read on the side stream
                if torch.is_tensor(t) and t.is_cuda:
                    t.record_stream(self.side)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.on:
            self._ctx.__exit__(*exc)
        return False

    def join(self, *outs):
        """The current stream waits for the side stream; returns `outs` (one or a tuple)."""
        if self.on:
            self.main.wait_stream(self.side)
            for t in outs:
                if torch.is_tensor(t) and t.is_cuda:
                    t.record_stream(self.main)
        return outs[0] if len(outs) == 1 else outs
