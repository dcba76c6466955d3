"""Test configuration: import paths and the `gpu` marker.

Layout on sys.path: the repo root (for `oracle`, test infrastructure only), the product tree
`e2e-parking-carla_amd/` (reference-named packages `model`, `tool`, `loss`, `trainer` and the
runtime `e2ep_amd`) and `tests/` (shared helpers)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "e2e-parking-carla_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libe2ep_hip.so")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
