"""Memory-safety checking for the e2ep ops (debug only; E2EP_GUARD=1 or install()).

Every device tensor the e2ep_amd op modules allocate is carved out of a larger buffer with
4 KiB canary regions before and after it, and (for torch.empty / empty_like) filled with
an all-ones bit pattern (NaN for fp32, -1 for integers) instead of whatever the allocator
hands back.  After every library call the stream is synchronised and every live canary is
verified, so a kernel that writes outside its buffers is named by the first call that
corrupts one, and a kernel that reads memory nobody wrote shows up as NaN downstream.
This mode is slow (a sync and a scan per call) and changes allocation patterns; it is a
test tool, never enabled on the product path.
"""
import sys
import weakref

import torch

GUARD_BYTES = 4096
_CANARY = 0xA5
_live = []  # (weakref to view, guard buffer, offset, nbytes)


class GuardError(RuntimeError):
    pass


def _guarded(shape, dtype, device, fill):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    dtype = dtype or torch.get_default_dtype()
    numel = 1
    for s in shape:
        numel *= int(s)
    esz = torch.empty((), dtype=dtype).element_size()
    nbytes = numel * esz
    buf = torch.full((nbytes + 2 * GUARD_BYTES,), _CANARY, dtype=torch.uint8, device=device)
    mid = buf[GUARD_BYTES:GUARD_BYTES + nbytes]
    mid.fill_(0 if fill == "zeros" else 0xFF)
    view = mid.view(dtype).view(tuple(int(s) for s in shape))
    _live.append((weakref.ref(view), buf, nbytes))
    return view


def _is_cuda(device, like=None):
    if device is None and like is not None:
        return like.is_cuda
    return device is not None and torch.device(device).type == "cuda"


class _TorchProxy:
    """Stands in for `torch` inside the op modules: guarded allocations, all else torch."""

    def __getattr__(self, name):
        return getattr(torch, name)

    def empty(self, *size, dtype=None, device=None, **kw):
        if not _is_cuda(device):
            return torch.empty(*size, dtype=dtype, device=device, **kw)
        return _guarded(size, dtype, device, "poison")

    def zeros(self, *size, dtype=None, device=None, **kw):
        if not _is_cuda(device):
            return torch.zeros(*size, dtype=dtype, device=device, **kw)
        return _guarded(size, dtype, device, "zeros")

    def empty_like(self, t, dtype=None, device=None, **kw):
        if not _is_cuda(device, t):
            return torch.empty_like(t, dtype=dtype, device=device, **kw)
        return _guarded(tuple(t.shape), dtype or t.dtype, device or t.device, "poison")

    def zeros_like(self, t, dtype=None, device=None, **kw):
        if not _is_cuda(device, t):
            return torch.zeros_like(t, dtype=dtype, device=device, **kw)
        return _guarded(tuple(t.shape), dtype or t.dtype, device or t.device, "zeros")


def check(after):
    """Verify every canary (synchronises); drop buffers whose tensor has died."""
    torch.cuda.synchronize()
    keep = []
    for ref, buf, nbytes in _live:
        head = buf[:GUARD_BYTES]
        tail = buf[GUARD_BYTES + nbytes:]
        bad_h = int((head != _CANARY).sum())
        bad_t = int((tail != _CANARY).sum())
        if bad_h or bad_t:
            raise GuardError(f"{after}: {bad_h} bytes before / {bad_t} bytes after a "
                             f"{nbytes}-byte buffer were overwritten")
        if ref() is not None:
            keep.append((ref, buf, nbytes))
    _live[:] = keep


_installed = False


def install():
    """Route the op modules' allocations through the guard and check after every call."""
    global _installed
    if _installed:
        return
    from . import _lib
    proxy = _TorchProxy()
    for name in ("e2ep_amd.conv", "e2ep_amd.nn_ops", "e2ep_amd.lss", "e2ep_amd.bev_stem",
                 "e2ep_amd.optim", "e2ep_amd.losses"):
        __import__(name)
        mod = sys.modules[name]
        if hasattr(mod, "torch"):
            mod.torch = proxy
    raw_call = _lib.call

    def call(name, *args):
        raw_call(name, *args)
        check(name)
    _lib.call = call
    _installed = True
