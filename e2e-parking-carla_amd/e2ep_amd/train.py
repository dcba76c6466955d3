"""Graph-captured training step for the ParkingModel (MI355X).

The reference steps through PyTorch-Lightning eagerly (trainer/pl_trainer.py:55-83 +
Adam at :116-121, DDP via pl_train.py:47).  Here one step — forward, the three losses,
backward and the Adam update — is captured once into HIP graphs and replayed, so the
~1,500 kernel launches of a step cost a few launches from the host.

Optimizer: e2ep_amd.optim.FlatAdam (one fused launch over a flat parameter buffer; the
gradients are read where autograd left them).

Data parallelism (one process per GPU, RCCL over xGMI): after backward the gradients are
gathered into one flat fp32 buffer (one launch), that buffer is all-reduced once per step
(sum; the 1/world mean is folded into the Adam launch — DistributedDataParallel's averaging,
without its per-bucket hooks), then the optimizer graph runs.  The all-reduce stays outside
the graphs.  bev_encoder.layer4 has no gradient (never run, reference
model/bev_encoder.py:21): callers freeze it so it is not part of the step.

Graph replay order per step: g_bwd (fwd + losses + bwd) -> [g_gather -> all-reduce] -> g_opt.
Graphs are captured through e2ep_amd.graphs.capture, which repairs memset nodes (they do
not replay correctly on this ROCm stack) before instantiation.
"""
import torch
import torch.distributed as dist

from . import graphs
from .optim import FlatAdam


class TrainStep:
    def __init__(self, module, batch, lr=1e-4, weight_decay=1e-4, world=1, graph=True,
                 warmup=3, optimizer=None):
        self.module = module
        self.batch = batch
        self.world = world
        self.graph = graph
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.opt = optimizer if optimizer is not None else FlatAdam(
            self.params, lr=lr, weight_decay=weight_decay)
        self.flat_grad = (torch.zeros(self.opt.numel, dtype=torch.float32,
                                      device=self.params[0].device) if world > 1 else None)
        self.loss = None
        self.g_bwd = self.g_gather = self.g_opt = None
        self._host_sync = world > 1 and dist.get_backend() == "gloo"
        if graph:
            self._capture(warmup)

    # -- pieces ---------------------------------------------------------------------------
    def _fwd_bwd(self):
        self.opt.zero_grad(set_to_none=True)  # autograd hands its gradient tensors over
        loss = self.module.training_step(self.batch, 0)
        loss.backward()
        return loss.detach()

    def _gather(self):
        if self.world > 1:
            self.opt.gather_grads(self.flat_grad)

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat_grad)

    def _update(self):
        if self.world > 1:
            self.opt.step(self.flat_grad, 1.0 / self.world)
        else:
            self.opt.step()

    def _eager(self):
        loss = self._fwd_bwd()
        self.opt.prepare()
        self._gather()
        self._allreduce()
        self._update()
        return loss

    # -- capture --------------------------------------------------------------------------
    def _capture(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.g_bwd, self.loss, self.memsets = graphs.capture(self._fwd_bwd)
        # the captured gradients keep their (graph-pool) addresses on every replay
        self.opt.prepare()
        if self.world > 1:
            self.g_gather, _, _ = graphs.capture(self._gather, pool=self.g_bwd.pool())
        self.g_opt, _, _ = graphs.capture(self._update, pool=self.g_bwd.pool())

    def __call__(self, batch=None):
        """One training step; `batch` (optional) is copied into the captured input buffers."""
        if batch is not None:
            for k, v in batch.items():
                if torch.is_tensor(v) and torch.is_tensor(self.batch.get(k)) and self.batch[k].is_cuda:
                    self.batch[k].copy_(v, non_blocking=True)
        if not self.graph:
            self.loss = self._eager()
            return self.loss
        self.g_bwd.replay()
        if self.world > 1:
            self.g_gather.replay()
            if self._host_sync:
                # gloo's CUDA all-reduce does not order itself after graph replays on this
                # stack (it hangs); RCCL's does.  Only the gloo rehearsal path pays this.
                torch.cuda.synchronize()
            self._allreduce()
        self.g_opt.replay()
        return self.loss
