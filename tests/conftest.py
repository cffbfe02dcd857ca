"""pytest setup: import paths and the `gpu` marker.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic of the C ABI
(config validation, plans, Poisson tables) and that libscgpu.so exports every symbol
include/scgpu.h declares. `-m gpu` runs on an MI355X: parity of the HIP kernels with the
oracle, called through the C ABI.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SCG_PKG_ROOT=exp/NAME: run the suite against an experiment build (tools/exp_build.py)
PKG_ROOT = os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd")
if not os.path.isabs(PKG_ROOT):
    PKG_ROOT = os.path.join(REPO, PKG_ROOT)
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels run)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
