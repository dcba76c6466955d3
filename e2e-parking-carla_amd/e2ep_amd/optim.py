"""Fused flat Adam for the ParkingModel train step (csrc/adam.hip).

The reference optimises with torch.optim.Adam(lr, weight_decay) over ~570 parameter
tensors (trainer/pl_trainer.py:116-121).  Stepping them tensor by tensor costs thousands
of small launches per step (and accumulating every gradient into a zeroed .grad another
~570).  Here all parameters live in ONE flat fp32 buffer (each nn.Parameter's storage is a
16-byte-aligned view into it), exp_avg / exp_avg_sq are flat buffers of the same layout,
and one launch steps everything, reading each gradient straight from the tensor autograd
produced (a device table of gradient addresses; .grad is set to None before backward so
autograd hands its result over without an accumulate).  For data parallelism the
gradients are gathered into a flat buffer of the same layout by one more launch, and
that buffer is what RCCL all-reduces.

state_dict() / load_state_dict() use torch.optim.Adam's format, so checkpoints move
between this optimizer and the reference's.
"""
import torch

from . import _lib

_ALIGN = 4  # elements (16 bytes)


class FlatAdam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.params = list(params)
        if not self.params:
            raise ValueError("FlatAdam: empty parameter list")
        dev = self.params[0].device
        if dev.type != "cuda":
            raise _lib.E2EPError("FlatAdam runs on a HIP device only")
        for p in self.params:
            if p.dtype != torch.float32 or p.device != dev:
                raise _lib.E2EPError("FlatAdam: parameters must be fp32 on one device")
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        lib = _lib.load()
        chunk = lib.e2ep_adam_chunk_elems()
        offs, rows, off = [], [], 0
        for i, p in enumerate(self.params):
            offs.append(off)
            n = p.numel()
            for s in range(0, n, chunk):
                rows.append((i, s, min(chunk, n - s), 0))
            off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                v = self.flat[o:o + p.numel()].view_as(p)
                v.copy_(p)
                p.data = v
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_count = torch.zeros(1, dtype=torch.float32, device=dev)
        self.offsets = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.chunks = torch.tensor(rows, dtype=torch.int32, device=dev).reshape(-1)
        self.n_chunks = len(rows)
        self._offs_host = offs
        self._gtab = torch.zeros(len(self.params), dtype=torch.int64, device=dev)
        self._gkey = None

    # -- gradients --------------------------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def prepare(self):
        """Point the device gradient table at the current .grad tensors (one small H2D copy,
        only when an address changed).  Call it outside graph capture."""
        key = []
        for p in self.params:
            g = p.grad
            if g is None:
                key.append(0)
                continue
            if g.dtype != torch.float32 or not g.is_contiguous() or g.device != self.flat.device:
                raise _lib.E2EPError("FlatAdam: gradients must be contiguous fp32 on the device")
            key.append(g.data_ptr())
        key = tuple(key)
        if key != self._gkey:
            if torch.cuda.is_current_stream_capturing():
                raise _lib.E2EPError("FlatAdam.prepare: gradient addresses changed during capture")
            self._gtab.copy_(torch.tensor(key, dtype=torch.int64))
            self._gkey = key

    def gather_grads(self, out):
        """Per-tensor gradients -> `out` (flat, parameter layout) for the all-reduce."""
        _lib.call("e2ep_grad_gather", _lib.ptr(self.chunks), self.n_chunks, _lib.ptr(self.offsets),
                  _lib.ptr(self._gtab), _lib.ptr(out), _lib.stream())

    # -- update -----------------------------------------------------------------------------
    def step(self, grad_flat=None, grad_scale=1.0):
        """One Adam step from the prepared gradient table, or from `grad_flat` (scaled by
        grad_scale, e.g. 1/world for an all-reduced sum)."""
        if grad_flat is None and self._gkey is None:
            raise _lib.E2EPError("FlatAdam.step: call prepare() after backward")
        b1, b2 = self.betas
        _lib.call("e2ep_adam_step", _lib.ptr(self.chunks), self.n_chunks, _lib.ptr(self.offsets),
                  None if grad_flat is not None else _lib.ptr(self._gtab),
                  _lib.ptr(grad_flat) if grad_flat is not None else None,
                  _lib.ptr(self.flat), _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq),
                  _lib.ptr(self.step_count), float(self.lr), float(b1), float(b2), float(self.eps),
                  float(self.weight_decay), float(grad_scale), _lib.stream())

    # -- torch.optim.Adam-format state --------------------------------------------------------
    def state_dict(self):
        state = {}
        for i, (p, o) in enumerate(zip(self.params, self._offs_host)):
            n = p.numel()
            state[i] = {"step": self.step_count[0].detach().cpu().clone(),
                        "exp_avg": self.exp_avg[o:o + n].view_as(p).clone(),
                        "exp_avg_sq": self.exp_avg_sq[o:o + n].view_as(p).clone()}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps,
                 "weight_decay": self.weight_decay, "amsgrad": False, "maximize": False,
                 "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.params)))}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        g = sd["param_groups"][0]
        self.lr, self.betas, self.eps, self.weight_decay = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        steps = set()
        with torch.no_grad():
            for i, (p, o) in enumerate(zip(self.params, self._offs_host)):
                s = sd["state"].get(i)
                if s is None:
                    continue
                n = p.numel()
                self.exp_avg[o:o + n].copy_(s["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
                steps.add(float(s["step"]))
        if len(steps) > 1:
            raise ValueError("FlatAdam keeps one step count; the state has several")
        self.step_count.fill_(steps.pop() if steps else 0.0)
