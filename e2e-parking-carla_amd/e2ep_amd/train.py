"""Graph-captured training step for the ParkingModel (MI355X).

The reference steps through PyTorch-Lightning eagerly (trainer/pl_trainer.py:55-83 +
Adam at :116-121, DDP via pl_train.py:47).  Here one step — zero grads, forward, the three
losses, backward and the Adam update — is captured once into a HIP graph and replayed, so
the ~1,500 kernel launches of a step cost one launch from the host.

Data parallelism (one process per GPU, RCCL over xGMI): gradients live in ONE flat fp32
buffer (every parameter's .grad is a view into it), so the exchange is a single RCCL
all-reduce of 78 MB per step between the captured backward graph and the captured optimizer
graph; the loss is pre-scaled by 1/world so the all-reduce sum is the mean gradient
(DistributedDataParallel semantics, without its per-bucket hooks).  bev_encoder.layer4 has
no gradient (never run, reference model/bev_encoder.py:21) and is left out of the buffer.
"""
import torch
import torch.distributed as dist


class TrainStep:
    def __init__(self, module, batch, lr=1e-4, weight_decay=1e-4, world=1, graph=True,
                 warmup=3):
        self.module = module
        self.batch = batch
        self.world = world
        self.graph = graph
        self.params = [p for p in module.parameters() if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.opt = torch.optim.Adam(self.params, lr=lr, weight_decay=weight_decay,
                                    capturable=graph, foreach=True)
        self.scale = 1.0 / world
        self.loss = None
        self.g_bwd = self.g_opt = None
        if graph:
            self._capture(warmup)

    # -- eager pieces ---------------------------------------------------------------------
    def _fwd_bwd(self):
        self.flat_grad.zero_()
        loss = self.module.training_step(self.batch, 0)
        (loss * self.scale if self.world > 1 else loss).backward()
        return loss.detach()

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat_grad)

    # -- capture --------------------------------------------------------------------------
    def _capture(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._fwd_bwd()
                self._allreduce()
                self.opt.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.g_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_bwd):
            self.loss = self._fwd_bwd()
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, pool=self.g_bwd.pool()):
            self.opt.step()

    def __call__(self, batch=None):
        """One training step; `batch` (optional) is copied into the captured input buffers."""
        if batch is not None:
            for k, v in batch.items():
                if torch.is_tensor(v) and torch.is_tensor(self.batch.get(k)) and self.batch[k].is_cuda:
                    self.batch[k].copy_(v, non_blocking=True)
        if not self.graph:
            self.loss = self._fwd_bwd()
            self._allreduce()
            self.opt.step()
            return self.loss
        self.g_bwd.replay()
        self._allreduce()
        self.g_opt.replay()
        return self.loss
