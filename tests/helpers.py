"""Shared test helpers: golden loading, tolerance checks, weight/batch construction."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


def rel_l2(a, b):
    a = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a.detach().cpu()).double()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b.detach().cpu()).double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def max_scaled(a, b):
    """max|a-b| / max|b| — the max-scaled form of the 1e-4 contract."""
    a = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a.detach().cpu()).double()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b.detach().cpu()).double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def reference_state(model, seed=1234):
    from weights import make_state
    return make_state(model.state_dict(), seed)
