"""Graph-captured training step for the ParkingModel (MI355X).

The reference steps through PyTorch-Lightning eagerly (trainer/pl_trainer.py:55-83 +
Adam at :116-121, DDP via pl_train.py:47).  Here one step — forward, the three losses,
backward and the Adam update — is captured once into HIP graphs and replayed, so the
~1,500 kernel launches of a step cost a few launches from the host.

Optimizer: e2ep_amd.optim.FlatAdam (one fused launch over a flat parameter buffer; the
gradients are read where autograd left them).  Its learning rate is a device scalar that
__call__ refreshes from param_groups[0]['lr'] before each replay, so an LR scheduler
(the reference's CosineAnnealingLR) acts on the captured step.

Data parallelism (one process per GPU, RCCL over xGMI; DistributedDataParallel semantics
without its module wrapper), one flat fp32 gradient buffer in FlatAdam's layout; the
1/world mean is folded into the Adam launch.
  * graph mode (the bench at N > 1): the backward runs in two segments
    (e2ep_amd.segments; the model cuts its forward below the BEV encoder): g_s1 (fwd + losses
    + stage-1 backward: heads, transformer, BEV encoder) -> g_s1g (their gradients -> the flat
    buffer) -> the host issues the stage-1 buckets' all-reduces (~25 MB each, reverse layout
    order) on a communication stream -> g_s2 (stage 2: lift-splat + camera encoder backward,
    concurrent with those all-reduces) -> g_s2g -> the stage-2 bucket(s) -> the compute stream
    waits for every bucket -> g_opt.  With gloo and device tensors (the one-GPU rehearsal of
    this path) the same graphs and bucket ranges run, each bucket staged through pinned host
    memory: after g_s1g the comm stream copies the stage-1 buckets out, g_s2 is replayed, the
    host waits for those copies only, all-reduces the buckets on the host (while stage 2 runs
    on the GPU) and the comm stream copies them back; then the same for stage 2.  No
    collective is captured: on this stack (torch 2.10 /
    RCCL 2.26) a captured ProcessGroupNCCL collective made the c10d watchdog fault on its
    capture-time event, and a backward graph with bucket gathers forked onto a side stream
    replayed wrong camera-encoder gradients (profiles/r02/ddp_diag/); here every
    collective is an ordinary host-issued RCCL call between graph replays.
  * graph mode without cut points (or segment=False): g_bwd (fwd + losses + bwd) -> g_gather -> ONE
    all-reduce of the flat buffer issued from the host between the replays -> g_opt.
  * eager mode: DDP-style overlap — the buffer is cut into ~25 MB buckets in reverse layout
    order; a post-accumulate-grad hook per parameter counts arrivals and, when a bucket is
    complete (and every earlier one issued: the same order on every rank), a side stream
    waits on an event of the forward/backward stream, gathers the bucket and all-reduces
    it asynchronously while backward continues.
  * gloo with device tensors (the one-GPU rehearsal): gloo does not order itself against
    HIP streams, so the flat buffer is staged explicitly through pinned host memory (copy,
    the host waits for the stream, all-reduce on the host, copy back).

Graphs are captured through e2ep_amd.graphs.capture, which repairs memset nodes (they do
not replay correctly on this ROCm stack) before instantiation.

Graph mode captures the lift-splat pillar plan of the batch's rig, planned before the capture
with the reference's fp32 host algebra whether the rig arrives as host or device tensors
(BevModel.prepare_capture; the plans are kept alive with the graphs): a later batch with a
different intrinsics/extrinsics rig raises instead of silently training on the captured plan
(the CARLA rig is constant).
"""
import os

import torch
import torch.distributed as dist

from . import _lib, graphs, segments
from .optim import FlatAdam

BUCKET_MB = 25.0  # DistributedDataParallel's default bucket_cap_mb


def _rig_key(batch):
    """The rig's shapes and fp32 bytes (a device rig is copied to the host: one small
    synchronising copy, only when a batch is handed to a graph-mode step)."""
    k, e = batch.get("intrinsics"), batch.get("extrinsics")
    if not (torch.is_tensor(k) and torch.is_tensor(e)):
        return None
    k, e = k.detach().float().cpu().contiguous(), e.detach().float().cpu().contiguous()
    return (tuple(k.shape), tuple(e.shape), k.numpy().tobytes(), e.numpy().tobytes())


class GradBuckets:
    """Bucketed, hook-driven gradient all-reduce over the optimizer's flat layout.

    `opt` supplies `spans` ([(flat offset, numel)] per parameter, in layout order),
    `gather_grads(out, params=(i0, i1))` and `prepare(params=(i0, i1))` (point the device
    gradient table at the current .grad tensors of that range)."""

    def __init__(self, params, opt, flat, bucket_mb=BUCKET_MB):
        self.params, self.opt, self.flat = params, opt, flat
        self.cuda = flat.is_cuda
        cap = int(bucket_mb * 2 ** 20) // 4
        spans = opt.spans
        self.buckets = []  # (i0, i1, lo, hi): parameters [i0, i1), flat [lo, hi)
        i1 = len(params)
        while i1 > 0:
            i0, n = i1, 0
            while i0 > 0 and (n == 0 or n + spans[i0 - 1][1] <= cap):
                i0 -= 1
                n += spans[i0][1]
            lo = spans[i0][0]
            hi = flat.numel() if i1 == len(params) else spans[i1][0]  # include alignment pad
            self.buckets.append((i0, i1, lo, hi))
            i1 = i0
        self.of = {}
        for b, (i0, i1, _, _) in enumerate(self.buckets):
            for i in range(i0, i1):
                self.of[i] = b
        self.comm = torch.cuda.Stream(device=flat.device) if self.cuda else None
        self.has = torch.zeros(len(params), dtype=torch.int64, device=flat.device)
        self.active = False
        self._handles = [p.register_post_accumulate_grad_hook(self._hook_for(i))
                         for i, p in enumerate(params)]

    def _hook_for(self, i):
        def hook(_p):
            if self.active:
                self._arrived(i)
        return hook

    def arm(self):
        """Start a step.  Called on the thread and stream that run forward/backward: the hooks
        run on autograd's device thread, whose current stream inside a hook need not be the
        stream the gradient kernels were issued on (under capture it can be a stream outside
        the capture), so the bucket fork waits on an event of THIS stream."""
        self.pending = [i1 - i0 for (i0, i1, _, _) in self.buckets]
        self.streams = [[] for _ in self.buckets]  # non-main streams gradients arrived on
        self.next = 0
        self.works = []
        self.active = True
        if self.cuda:
            self.main = torch.cuda.current_stream()
            self.capturing = torch.cuda.is_current_stream_capturing()

    def _arrived(self, i):
        b = self.of[i]
        if self.cuda and not self.capturing:
            # the stream this gradient was produced on (a model branch's side stream for the
            # segmentation / depth heads): the bucket's gather waits for every one of them,
            # not only for the stream of the hook that completes the bucket
            here = torch.cuda.current_stream()
            if here != self.main and all(here != s for s in self.streams[b]):
                self.streams[b].append(here)
        self.pending[b] -= 1
        while self.next < len(self.buckets) and self.pending[self.next] == 0:
            self._launch(self.next)
            self.next += 1

    def _launch(self, b):
        i0, i1, lo, hi = self.buckets[b]
        if not self.cuda:
            self.opt.prepare(params=(i0, i1))
            self.opt.gather_grads(self.flat, params=(i0, i1))
            self.works.append(dist.all_reduce(self.flat[lo:hi], async_op=True))
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.comm.wait_event(ev)
        for st in self.streams[b]:  # eager: every stream a gradient of the bucket came from
            ev2 = torch.cuda.Event()
            ev2.record(st)
            self.comm.wait_event(ev2)
        with torch.cuda.stream(self.comm):
            if not self.capturing:
                self.opt.prepare(params=(i0, i1))  # fresh gradient addresses (eager)
            self.opt.gather_grads(self.flat, params=(i0, i1))
            self.works.append(dist.all_reduce(self.flat[lo:hi], async_op=True))

    def finish(self):
        """Issue the buckets whose tensors had no gradient this step (zeros), in order, and
        make the compute stream wait for every all-reduce."""
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        for w in self.works:
            w.wait()
        if self.cuda:
            self.main.wait_stream(self.comm)
        self.opt.prepare()
        self.opt.has_grad(self.has)
        dist.all_reduce(self.has, op=dist.ReduceOp.MAX)
        self.works = []
        self.active = False


class TrainStep:
    def __init__(self, module, batch, lr=1e-4, weight_decay=1e-4, world=1, graph=True,
                 warmup=3, optimizer=None, bucket_mb=BUCKET_MB, overlap=None, ddp=None,
                 segment=True):
        self.module = module
        self.batch = batch
        self.world = world
        # ddp: run the exchange (default: world > 1; ddp=True at world 1 exercises the
        # collective path on one device, e.g. RCCL capture in tests)
        self.ddp = world > 1 if ddp is None else bool(ddp)
        self.graph = graph
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.opt = optimizer if optimizer is not None else FlatAdam(
            self.params, lr=lr, weight_decay=weight_decay)
        dev = self.params[0].device
        self.flat_grad = (torch.zeros(self.opt.numel, dtype=torch.float32, device=dev)
                          if self.ddp else None)
        # which parameters had a gradient on ANY rank (all-reduced MAX with the gradients):
        # every replica steps the same set, as under DDP (a rank-local mask lets
        # replicas drift when a branch is rank-dependent)
        self.has_grad = (torch.zeros(len(self.params), dtype=torch.int64, device=dev)
                         if self.ddp else None)
        self.backend = dist.get_backend() if self.ddp else None
        if overlap is None:
            overlap = os.environ.get("E2EP_DDP_OVERLAP", "1") != "0"
        # hook-driven bucket all-reduce overlapping backward: eager steps with RCCL, and host
        # tensors (gloo on CPU); never inside a captured graph (module docstring)
        self._bucket_mb = bucket_mb
        self.overlap = bool(self.ddp and overlap and not graph and
                            (self.backend == "nccl" or not self.flat_grad.is_cuda))
        self.buckets = (GradBuckets(self.params, self.opt, self.flat_grad, bucket_mb)
                        if self.overlap else None)
        if self.buckets is not None:
            self.has_grad = self.buckets.has
        self._host = (torch.empty(self.opt.numel, dtype=torch.float32, pin_memory=True)
                      if self.ddp and self.backend != "nccl" and not self.overlap
                      and self.flat_grad.is_cuda else None)
        self.loss = None
        self.g_bwd = self.g_gather = self.g_opt = None
        # segmented backward (graph mode; RCCL, or gloo staged through self._host): stage
        # graphs, their gathers, bucket ranges.  segment=False keeps one backward graph.
        self.segmented = bool(segment and self.ddp and graph and
                              (self.backend == "nccl" or self._host is not None))
        self.g_s1 = self.g_s1g = self.g_s2 = self.g_s2g = None
        self.seg_buckets = None  # ([stage-1 (lo, hi)], [stage-2 (lo, hi)]) of the flat buffer
        self._rig = _rig_key(batch)
        # test-only: (stage, bucket index) of a segmented-exchange bucket whose all-reduce is
        # skipped (tests/test_ddp_gpu.py proves the parity check fails without it)
        self._test_skip = None
        self._plans = []
        if graph:
            # plan every rig the capture will meet outside it (host algebra, bit-exact), and
            # keep those plans as long as the graphs that read them
            self._plans = [m.prepare_capture(batch) for m in module.modules()
                           if hasattr(m, "prepare_capture")]
            self._capture(warmup)

    # -- pieces ---------------------------------------------------------------------------
    def _fwd_bwd(self):
        self.opt.zero_grad(set_to_none=True)  # autograd hands its gradient tensors over
        if self.buckets is not None:
            self.buckets.arm()
        loss = self.module.training_step(self.batch, 0)
        # the seed gradient: a persistent ones scalar (loss.backward() would fill one per step)
        if getattr(self, "_one", None) is None or self._one.device != loss.device:
            self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
        loss.backward(self._one)
        if self.buckets is not None:
            self.buckets.finish()
        return loss.detach()

    def _gather(self):
        if self.ddp and self.buckets is None:
            self.opt.gather_grads(self.flat_grad)
            self.opt.has_grad(self.has_grad)

    def _allreduce(self):
        """Non-overlapped exchange (gloo): host-staged for device tensors, with the ordering
        explicit — the host waits for the compute stream before gloo reads the copy."""
        if not self.ddp or self.buckets is not None:
            return
        if self._host is None:
            dist.all_reduce(self.flat_grad)
            dist.all_reduce(self.has_grad, op=dist.ReduceOp.MAX)
            return
        self._host.copy_(self.flat_grad, non_blocking=True)
        has = self.has_grad.cpu()  # synchronises the stream too
        torch.cuda.current_stream().synchronize()
        dist.all_reduce(self._host)
        dist.all_reduce(has, op=dist.ReduceOp.MAX)
        self.flat_grad.copy_(self._host, non_blocking=True)
        self.has_grad.copy_(has, non_blocking=True)

    def _update(self):
        if self.ddp:
            self.opt.step(self.flat_grad, 1.0 / self.world, has_grad=self.has_grad)
        else:
            self.opt.step()

    def _eager(self):
        loss = self._fwd_bwd()
        self.opt.prepare()
        self._gather()
        self._allreduce()
        self._update()
        return loss

    # -- segmented backward (graph mode with RCCL) ----------------------------------------
    def _stage1(self):
        self.opt.zero_grad(set_to_none=True)
        with segments.record() as rec:
            loss = self.module.training_step(self.batch, 0)
        self._pairs = rec.pairs
        loss.backward()
        return loss.detach()

    def _stage2(self):
        segments.backward_rest(self._pairs)

    def _buckets_of(self, i0, i1, bucket_mb):
        """Flat ranges of ~bucket_mb over parameters [i0, i1), last parameters first (the
        order their gradients complete in, as DistributedDataParallel buckets them)."""
        cap = int(bucket_mb * 2 ** 20) // 4
        spans, out = self.opt.spans, []
        end = self.opt.numel if i1 == len(self.params) else spans[i1][0]
        j1 = i1
        while j1 > i0:
            j0, n = j1, 0
            while j0 > i0 and (n == 0 or n + spans[j0 - 1][1] <= cap):
                j0 -= 1
                n += spans[j0][1]
            lo = spans[j0][0]
            out.append((lo, end))
            end, j1 = lo, j0
        return out

    def _capture_segmented(self, bucket_mb):
        """Capture g_s1 / g_s1g / g_s2 / g_s2g; False (nothing kept) when the module declares
        no cut point or its stage-1 gradients are not a suffix of the flat layout."""
        segments.ensure_anchor(self.params[0].device)
        g1, loss, _ = graphs.capture(self._stage1)
        if not self._pairs:
            return False
        has1 = [p.grad is not None for p in self.params]
        if not any(has1):
            return False
        i1 = has1.index(True)
        if not all(has1[i1:]):
            return False
        self.opt.prepare(params=(i1, len(self.params)))
        g1g, _, _ = graphs.capture(lambda: self.opt.gather_grads(self.flat_grad,
                                                                 params=(i1, len(self.params))),
                                   pool=g1.pool())
        marks = segments.grad_marks(self.params[i1:])
        g2, _, _ = graphs.capture(self._stage2, pool=g1.pool())
        if not segments.stage2_leaves_stage1(self.params[i1:], marks):
            return False  # a parameter on both sides of the cut: one backward graph instead
        self.opt.prepare()
        if i1 > 0:
            g2g, _, _ = graphs.capture(lambda: self.opt.gather_grads(self.flat_grad, params=(0, i1)),
                                       pool=g1.pool())
        else:
            g2g = None
        self.g_s1, self.g_s1g, self.g_s2, self.g_s2g, self.loss = g1, g1g, g2, g2g, loss
        self.seg_buckets = (self._buckets_of(i1, len(self.params), bucket_mb),
                            self._buckets_of(0, i1, bucket_mb))
        self.comm = torch.cuda.Stream(device=self.flat_grad.device)
        # which tensors have a gradient is fixed by the captured graphs: all-reduced once (MAX)
        self.opt.has_grad(self.has_grad)
        if self._host is None:
            dist.all_reduce(self.has_grad, op=dist.ReduceOp.MAX)
        else:
            has = self.has_grad.cpu()  # synchronises the stream
            dist.all_reduce(has, op=dist.ReduceOp.MAX)
            self.has_grad.copy_(has)
        return True

    def _replay_segmented(self):
        if self._host is not None:
            self._replay_segmented_host()
            return
        main = torch.cuda.current_stream()
        works = []

        def issue(stage, ranges):
            ev = torch.cuda.Event()
            ev.record(main)
            self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                for j, (lo, hi) in enumerate(ranges):
                    if self._test_skip != (stage, j):
                        works.append(dist.all_reduce(self.flat_grad[lo:hi], async_op=True))

        self.g_s1.replay()
        self.g_s1g.replay()
        issue(0, self.seg_buckets[0])  # overlaps the stage-2 backward below
        self.g_s2.replay()
        if self.g_s2g is not None:
            self.g_s2g.replay()
        issue(1, self.seg_buckets[1])
        for w in works:
            w.wait()  # the compute stream waits for every bucket
        self.g_opt.replay()

    def _replay_segmented_host(self):
        """_replay_segmented for gloo with device tensors: the same graphs and bucket ranges,
        each bucket staged through the pinned host buffer.  The comm stream copies a stage's
        buckets out after its gather graph, the host waits for those copies only, all-reduces
        the buckets on the host while the GPU runs on, and the comm stream copies them back;
        the compute stream waits for the comm stream before the optimizer graph."""
        main = torch.cuda.current_stream()
        h, flat = self._host, self.flat_grad

        def copy_out(ranges):
            ev = torch.cuda.Event()
            ev.record(main)
            self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                for lo, hi in ranges:
                    h[lo:hi].copy_(flat[lo:hi], non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.comm)
            return done

        def exchange(stage, ranges, done):
            done.synchronize()  # the host waits for this stage's copies, not for the GPU
            works = [dist.all_reduce(h[lo:hi], async_op=True)
                     for j, (lo, hi) in enumerate(ranges) if self._test_skip != (stage, j)]
            for w in works:
                w.wait()
            with torch.cuda.stream(self.comm):
                for lo, hi in ranges:
                    flat[lo:hi].copy_(h[lo:hi], non_blocking=True)

        self.g_s1.replay()
        self.g_s1g.replay()
        d1 = copy_out(self.seg_buckets[0])
        self.g_s2.replay()  # stage 2 on the GPU while the host exchanges stage 1
        exchange(0, self.seg_buckets[0], d1)
        if self.g_s2g is not None:
            self.g_s2g.replay()
        exchange(1, self.seg_buckets[1], copy_out(self.seg_buckets[1]))
        main.wait_stream(self.comm)
        self.g_opt.replay()

    # -- capture --------------------------------------------------------------------------
    def _capture(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.segmented:
            self.segmented = self._capture_segmented(self._bucket_mb)
            if self.segmented:
                self.g_opt, _, _ = graphs.capture(self._update, pool=self.g_s1.pool())
                return
            self.opt.zero_grad(set_to_none=True)
            self._pairs = None
        self.g_bwd, self.loss, self.memsets = graphs.capture(self._fwd_bwd)
        # the captured gradients keep their (graph-pool) addresses on every replay
        self.opt.prepare()
        if self.ddp and self.buckets is None:
            self.g_gather, _, _ = graphs.capture(self._gather, pool=self.g_bwd.pool())
        self.g_opt, _, _ = graphs.capture(self._update, pool=self.g_bwd.pool())

    def __call__(self, batch=None):
        """One training step; `batch` (optional) is copied into the captured input buffers."""
        if batch is not None:
            if self.graph and _rig_key(batch) != self._rig:
                raise _lib.E2EPError(
                    "TrainStep(graph=True) captured the lift-splat plan of the first batch's "
                    "camera rig; this batch has different intrinsics/extrinsics (build a new "
                    "TrainStep, or use graph=False, which plans every batch's rig)")
            for k, v in batch.items():
                if torch.is_tensor(v) and torch.is_tensor(self.batch.get(k)) and self.batch[k].is_cuda:
                    self.batch[k].copy_(v, non_blocking=True)
        sync_lr = getattr(self.opt, "sync_lr", None)
        if sync_lr is not None:
            sync_lr()
        if not self.graph:
            self.loss = self._eager()
            return self.loss
        if self.segmented:
            self._replay_segmented()
            return self.loss
        self.g_bwd.replay()
        if self.g_gather is not None:
            self.g_gather.replay()
            self._allreduce()
        self.g_opt.replay()
        return self.loss
