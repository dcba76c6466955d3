"""HIP-event timing of individual kernel launches, on the stream each kernel runs on.

bench.py enables it for a few eager steps right after its timed (graph-replayed) region to
measure the dominant kernel's average launch duration live (the `roofline.achieved`
figure); it is off by default and then costs one boolean test per launch.  Never enable it
while a step is being captured into a HIP graph."""
import os
from collections import defaultdict
from contextlib import contextmanager

import torch

_enabled = False
_events = defaultdict(list)
_work = defaultdict(float)


def detail():
    """Per-shape region names (E2EP_TIMING_DETAIL=1), for breakdown scripts only."""
    return _enabled and os.environ.get("E2EP_TIMING_DETAIL") == "1"


def name(kind, shape, tag=""):
    """Region name: `kind`, or `kind(shape)tag` under E2EP_TIMING_DETAIL=1."""
    return f"{kind}{tuple(shape)}{tag}" if detail() else kind


def enable(flag=True):
    global _enabled
    _enabled = flag


def reset():
    _events.clear()
    _work.clear()


@contextmanager
def region(name, work=0.0):
    """Time the launches enqueued inside; `work` = the launch's algorithmic FLOPs (or bytes),
    summed per region name for roofline figures."""
    if not _enabled:
        yield
        return
    _work[name] += float(work)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()  # records on torch's current stream == the stream the kernel is enqueued on
    try:
        yield
    finally:
        e.record()
        _events[name].append((s, e))


def summary():
    """{name: (launches, mean_ms, total_ms)} — synchronises."""
    torch.cuda.synchronize()
    out = {}
    for k, evs in _events.items():
        t = [s.elapsed_time(e) for s, e in evs]
        out[k] = (len(t), sum(t) / max(1, len(t)), sum(t))
    return out


def work():
    """{name: total algorithmic work recorded by region(..., work=)} since reset()."""
    return dict(_work)
