"""Shared test setup.

* registers the `gpu` marker: tests that launch HIP kernels (run on the MI355X box with `-m gpu`)
* puts the repo root (oracle/, bench helpers) and the package directory (drop-in `Pointcloud`, `PatchGeneration`,
  `pcd_native`) on sys.path -- the same way a reference notebook switches to this implementation.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


class ParityReport(UserWarning):
    """A measured parity figure (deviation percentiles, excluded fractions): issued as a warning so that it shows in
    pytest's warnings summary even for passing tests under -q (the round-end GPU run), and printed for -s."""


def report(msg: str):
    import warnings
    print(msg)
    warnings.warn(msg, ParityReport, stacklevel=2)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"))
    return load


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)
