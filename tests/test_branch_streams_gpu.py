"""Model branches on side streams (e2ep_amd.streams) under HIP-graph capture.

The camera depth head next to the feature head ("cam", reference model/cam_encoder.py:91-96)
and the segmentation head next to the control decoder ("heads", model/parking_model.py:60-69)
may run on side streams.  A weight-gradient fork (conv._Fork) taken from inside such a branch
made hipStreamEndCapture segfault (rounds 2 and 4); the fork is now never taken from a branch
stream.  Streams do not change any kernel's arithmetic, so the captured step with branches
gives the same parameters as the step without, bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(mod):
    return torch.cat([p.detach().reshape(-1) for p in mod.parameters()]).cpu()


@pytest.mark.parametrize("names", [("cam",), ("heads",), ("cam", "heads")])
def test_captured_step_with_branch_streams_equals_single_stream(names):
    from e2ep_amd import conv, streams
    from e2ep_amd.train import TrainStep
    from test_train_step_b8_gpu import _batch, _module
    assert conv.wgrad_overlap()  # weight-gradient forks on outside the branches
    runs = []
    for on in (set(names), set()):
        prev = streams.set_enabled(on)
        try:
            mod = _module()
            step = TrainStep(mod, _batch(), graph=True, warmup=2)
            losses = [float(step()) for _ in range(2)]
            torch.cuda.synchronize()
            runs.append((losses, _params(mod)))
            del step, mod
        finally:
            streams.set_enabled(prev)
    (l_on, p_on), (l_off, p_off) = runs
    assert l_on == l_off
    assert torch.equal(p_on, p_off)
