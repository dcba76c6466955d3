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

FlatAdam is a torch.optim.Optimizer with one param group, so the reference's
CosineAnnealingLR (trainer/pl_trainer.py:120) binds to it unchanged.  The learning rate the
kernel uses lives in a device fp64 scalar: step() (eager) and TrainStep (before each graph
replay) copy param_groups[0]['lr'] into it when the scheduler has changed it, so a captured
step follows the schedule.  betas / eps / weight_decay are fixed at construction (the
reference never changes them).

state_dict() / load_state_dict() use torch.optim.Adam's format, so checkpoints move
between this optimizer and the reference's.
"""
import torch

from . import _lib

_ALIGN = 4  # elements (16 bytes)


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        params = list(params)
        if not params:
            raise ValueError("FlatAdam: empty parameter list")
        if isinstance(params[0], dict):
            raise ValueError("FlatAdam: one parameter group only")
        dev = params[0].device
        if dev.type != "cuda":
            raise _lib.E2EPError("FlatAdam runs on a HIP device only")
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise _lib.E2EPError("FlatAdam: parameters must be fp32 on one device")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))
        self.params = self.param_groups[0]["params"]
        self.betas, self.eps, self.weight_decay = tuple(betas), eps, weight_decay
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
        # 1 for every tensor stepped at least once (written by the Adam kernel): state_dict
        # holds state for those only, as torch.optim.Adam does (a tensor that never had a
        # gradient, e.g. bev_encoder.layer4, has no state there)
        self.stepped = torch.zeros(len(self.params), dtype=torch.int32, device=dev)
        self.offsets = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.chunks = torch.tensor(rows, dtype=torch.int32, device=dev).reshape(-1)
        self.n_chunks = len(rows)
        self._offs_host = offs
        self.spans = [(o, p.numel()) for o, p in zip(offs, self.params)]
        self._gtab = torch.zeros(len(self.params), dtype=torch.int64, device=dev)
        self._has_bool = torch.zeros(len(self.params), dtype=torch.bool, device=dev)
        self._gkey = None
        # row range of each tensor in the chunk table (gradient buckets gather by rows)
        self.chunk_rows, r = [], 0
        for p in self.params:
            n = (p.numel() + chunk - 1) // chunk
            self.chunk_rows.append((r, r + n))
            r += n
        self.lr_dev = torch.full((1,), float(lr), dtype=torch.float64, device=dev)
        self._lr_written = float(lr)

    # -- learning rate ------------------------------------------------------------------------
    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    @lr.setter
    def lr(self, v):
        self.param_groups[0]["lr"] = v

    def sync_lr(self):
        """Copy param_groups[0]['lr'] (an LR scheduler's output) into the device scalar the
        Adam kernel reads, if it changed.  Not during capture: the kernel node reads the
        scalar at replay time, the host writes it between replays."""
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_written and not torch.cuda.is_current_stream_capturing():
            self.lr_dev.fill_(lr)
            self._lr_written = lr

    # -- gradients --------------------------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def prepare(self, params=None):
        """Point the device gradient table at the current .grad tensors (one small H2D copy,
        only when an address changed) — of all tensors, or of the index range `params` =
        (i0, i1) (one gradient bucket).  Call it outside graph capture."""
        i0, i1 = params if params is not None else (0, len(self.params))
        key = []
        for p in self.params[i0:i1]:
            g = p.grad
            if g is None:
                key.append(0)
                continue
            if g.dtype != torch.float32 or not g.is_contiguous() or g.device != self.flat.device:
                raise _lib.E2EPError("FlatAdam: gradients must be contiguous fp32 on the device")
            key.append(g.data_ptr())
        old = self._gkey if self._gkey is not None else (None,) * len(self.params)
        if tuple(key) != tuple(old[i0:i1]):
            if torch.cuda.is_current_stream_capturing():
                raise _lib.E2EPError("FlatAdam.prepare: gradient addresses changed during capture")
            self._gtab[i0:i1].copy_(torch.tensor(key, dtype=torch.int64))
            self._gkey = tuple(old[:i0]) + tuple(key) + tuple(old[i1:])

    def gather_grads(self, out, params=None):
        """Per-tensor gradients -> `out` (flat, parameter layout) for the all-reduce;
        `params` = (i0, i1) restricts it to one bucket of tensors."""
        if params is None:
            r0, r1 = 0, self.n_chunks
        else:
            r0, r1 = self.chunk_rows[params[0]][0], self.chunk_rows[params[1] - 1][1]
        if r1 <= r0:
            return
        import ctypes
        _lib.call("e2ep_grad_gather", ctypes.c_void_p(self.chunks.data_ptr() + 16 * r0), r1 - r0,
                  _lib.ptr(self.offsets), _lib.ptr(self._gtab), _lib.ptr(out), _lib.stream())

    # -- update -----------------------------------------------------------------------------
    @torch.no_grad()
    def has_grad(self, out):
        """out[i] = 1 if parameter i has a gradient this step (from the prepared table), else 0
        (int64, capturable).  Data-parallel callers all-reduce it with MAX and pass it to
        step(grad_flat, ..., has_grad=out): every replica then steps the same parameters."""
        torch.ne(self._gtab, 0, out=self._has_bool)
        out.copy_(self._has_bool)
        return out

    def step(self, grad_flat=None, grad_scale=1.0, closure=None, has_grad=None):
        """One Adam step from the prepared gradient table, or from `grad_flat` (scaled by
        grad_scale, e.g. 1/world for an all-reduced sum); tensors whose table entry is null
        (no gradient) are skipped either way.  With `grad_flat`, `has_grad` (int64 per
        parameter, non-zero = step it; see has_grad()) replaces this rank's own table, so a
        parameter that had a gradient on any rank is stepped on every rank, as under DDP.
        torch.optim-style calls (no arguments, or a closure) prepare the table themselves."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not torch.cuda.is_current_stream_capturing():
            self.prepare()
        self.sync_lr()
        b1, b2 = self.betas
        _lib.call("e2ep_adam_step", _lib.ptr(self.chunks), self.n_chunks, _lib.ptr(self.offsets),
                  _lib.ptr(has_grad if (has_grad is not None and grad_flat is not None)
                           else self._gtab),
                  _lib.ptr(grad_flat) if grad_flat is not None else None,
                  _lib.ptr(self.flat), _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq),
                  _lib.ptr(self.step_count), _lib.ptr(self.lr_dev), float(b1), float(b2),
                  float(self.eps), float(self.weight_decay), float(grad_scale),
                  _lib.ptr(self.stepped), _lib.stream())
        return loss

    # -- torch.optim.Adam-format state --------------------------------------------------------
    def state_dict(self):
        state = {}
        stepped = self.stepped.cpu().tolist()
        for i, (p, o) in enumerate(zip(self.params, self._offs_host)):
            if not stepped[i]:
                continue
            n = p.numel()
            state[i] = {"step": self.step_count[0].detach().cpu().clone(),
                        "exp_avg": self.exp_avg[o:o + n].view_as(p).clone(),
                        "exp_avg_sq": self.exp_avg_sq[o:o + n].view_as(p).clone()}
        group = {"lr": float(self.lr), "betas": self.betas, "eps": self.eps,
                 "weight_decay": self.weight_decay, "amsgrad": False, "maximize": False,
                 "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.params)))}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        g = sd["param_groups"][0]
        self.betas, self.eps, self.weight_decay = tuple(g["betas"]), g["eps"], g["weight_decay"]
        pg = self.param_groups[0]
        pg.update(lr=g["lr"], betas=self.betas, eps=self.eps, weight_decay=self.weight_decay)
        if "initial_lr" in g:
            pg["initial_lr"] = g["initial_lr"]
        steps = set()
        with torch.no_grad():
            self.stepped.zero_()
            for i, (p, o) in enumerate(zip(self.params, self._offs_host)):
                s = sd["state"].get(i)
                if s is None:
                    continue
                self.stepped[i] = 1
                n = p.numel()
                self.exp_avg[o:o + n].copy_(s["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
                steps.add(float(s["step"]))
        if len(steps) > 1:
            raise ValueError("FlatAdam keeps one step count; the state has several")
        self.step_count.fill_(steps.pop() if steps else 0.0)
