"""Fused HIP losses (csrc/loss.hip) vs the oracle restatement of the reference losses
(loss/control_loss.py, loss/seg_loss.py, loss/depth_loss.py) in fp64: values and input
gradients, with the edge cases the reference handles — PAD rows ignored (and the all-PAD
batch, NaN like torch), ignore-index 255 pixels counted in the plain mean, depth cells with
no return (all zeros) or out-of-range depth, and the hi-res 512^2 depth map (C4).
Tolerance: 1e-6 relative on values, rel-L2 1e-6 on gradients (fp32 kernels, fixed-order
reductions), and bitwise-identical results across two launches."""
import math

import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle():
    from oracle import parking_ref as O
    return O


def _gt_control(B, seed, pad_tail=True):
    g = torch.Generator().manual_seed(seed)
    gt = torch.randint(0, 200, (B, 15), generator=g)
    gt[:, 0], gt[:, 13], gt[:, 14] = 201, 202, 203
    if pad_tail:  # ragged sequences: some rows end early
        gt[0, 9:] = 203
        gt[B - 1, 5:] = 203
    return gt


@pytest.mark.parametrize("B", [1, 8, 64])
def test_control_ce_matches_reference(B):
    from e2ep_amd import losses
    O = _oracle()
    g = torch.Generator().manual_seed(B)
    pred = torch.randn(B, 14, 204, generator=g) * 3
    gt = _gt_control(B, B)
    ref_in = pred.double().requires_grad_()
    ref = O.control_loss(ref_in, gt)
    ref.backward()
    x = pred.to(DEV).requires_grad_()
    out = losses.control_ce(x, gt.to(DEV), 203)
    out.backward()
    assert abs(float(out) / float(ref) - 1) < 1e-6
    assert rel_l2(x.grad, ref_in.grad) < 1e-6
    out2 = losses.control_ce(pred.to(DEV), gt.to(DEV), 203)
    assert torch.equal(out2, out.detach())


def test_control_ce_all_pad_is_nan_like_torch():
    from e2ep_amd import losses
    gt = torch.full((2, 15), 203)
    out = losses.control_ce(torch.randn(2, 14, 204, device=DEV), gt.to(DEV), 203)
    assert math.isnan(float(out))


@pytest.mark.parametrize("B,hw", [(2, 200), (8, 200), (3, 37)])
def test_seg_weighted_ce_matches_reference(B, hw):
    from e2ep_amd import losses
    O = _oracle()
    g = torch.Generator().manual_seed(hw + B)
    pred = torch.randn(B, 1, 3, hw, hw, generator=g) * 2
    tgt = torch.randint(0, 3, (B, 1, hw, hw), generator=g)
    tgt[0, 0, :5, :7] = 255  # ignored pixels: 0 in the mean, still counted
    ref_in = pred.double().requires_grad_()
    ref = O.segmentation_loss(ref_in, tgt)
    ref.backward()
    x = pred.to(DEV).requires_grad_()
    out = losses.seg_weighted_ce(x, tgt.to(DEV), torch.tensor([1.0, 2.0, 2.0]))
    out.backward()
    assert abs(float(out) / float(ref) - 1) < 1e-6
    assert rel_l2(x.grad, ref_in.grad) < 1e-6
    assert float(x.grad[0, 0, :, :5, :7].abs().max()) == 0.0


@pytest.mark.parametrize("B,N,H", [(2, 4, 256), (8, 4, 256), (1, 6, 512)])
def test_depth_bce_matches_reference(B, N, H):
    from e2ep_amd import losses
    O = _oracle()
    g = torch.Generator().manual_seed(B * N + H)
    D = 48
    prob = torch.randn(B * N, D, H // 8, H // 8, generator=g).softmax(1)
    depth = torch.rand(B, N, H, H, generator=g) * 15.0
    depth[0, 0, :16, :16] = 0.0           # no return: background cells
    depth[0, 1, 8:16, :] = 40.0           # beyond the last bin: background
    depth[-1, -1, :8, :8] = 0.25          # exactly on the first bin edge: bin 0 -> background
    depth[-1, -1, :8, 8:16] = 0.5         # first foreground bin
    ref_in = prob.double().requires_grad_()
    ref = O.depth_loss(ref_in, depth.double())
    ref.backward()
    x = prob.to(DEV).requires_grad_()
    out = losses.depth_bce(x, depth.to(DEV), (0.5, 12.5, 0.25), 8)
    out.backward()
    assert abs(float(out) / float(ref) - 1) < 1e-6
    assert rel_l2(x.grad, ref_in.grad) < 1e-6
    # labels: the reference's own one-hot helper on the same depth map
    lab = losses.depth_onehot(depth, (0.5, 12.5, 0.25), 8)
    assert torch.equal(lab, O.depth_labels(depth))


def test_depth_bce_float64_depth_bins_in_float64():
    """The reference dataset yields float64 metres (dataset/carla_dataset.py:107-113), so the
    reference bins them in float64: a depth 1e-9 below a bin edge falls in the lower bin, while
    its fp32 rounding lands on the edge (upper bin).  The fp64 entry point must follow float64."""
    from e2ep_amd import losses
    O = _oracle()
    g = torch.Generator().manual_seed(7)
    prob = torch.randn(2, 48, 32, 32, generator=g).softmax(1)
    depth = torch.rand(1, 2, 256, 256, generator=g, dtype=torch.float64) * 15.0
    depth[0, 0, :8, :8] = 0.75 - 1e-9   # fp64: bin 1; fp32 rounds to 0.75: bin 2
    depth[0, 1, :8, :8] = 3.0 - 1e-10
    ref_in = prob.double().requires_grad_()
    ref = O.depth_loss(ref_in, depth)
    ref.backward()
    x = prob.to(DEV).requires_grad_()
    out = losses.depth_bce(x, depth.to(DEV), (0.5, 12.5, 0.25), 8)
    out.backward()
    assert abs(float(out) / float(ref) - 1) < 1e-6
    assert rel_l2(x.grad, ref_in.grad) < 1e-6
    out32 = losses.depth_bce(prob.to(DEV), depth.float().to(DEV), (0.5, 12.5, 0.25), 8)
    assert float(out32) != float(out)   # the fp32 path bins the edge cells differently
