"""The position steps' device arithmetic is the host build's, bit for bit (and the host build is the reference's:
tests/test_capi.py pins inv3_ref against torch.linalg.inv_ex, tests/test_oracle_golden.py the solve steps against
the reference's own output).  Random bunny-scale inputs: coordinates with full mantissas, where an operation-order
difference would show (fandisk's coordinates are short decimals)."""
import numpy as np
import pytest
import torch

import pcd_native as nat

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["edge", "feature", "corner", "flat", "new"])
def test_device_steps_equal_host_build(gpu, kind):
    rng = np.random.default_rng(5)
    n, m, k = 20000, 5000, 8
    pos = (rng.normal(size=(n, 3)) * 0.05 + np.array([0.03, 0.11, -0.02])).astype(np.float32)
    nrm = rng.normal(size=(n, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    ev = rng.normal(size=(n, 3)).astype(np.float32)
    ev /= np.linalg.norm(ev, axis=1, keepdims=True)
    ci = rng.choice(n, m, replace=False).astype(np.int64)
    nbr = rng.integers(0, n, (m, k)).astype(np.int64)
    nbr[:, 0] = ci
    K = {"edge": nat.STEP_EDGE, "feature": nat.STEP_FEATURE, "corner": nat.STEP_CORNER, "flat": nat.STEP_FLAT,
         "new": nat.STEP_NEW}[kind]
    d, alpha = 1e6, 0.2
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    off = torch.arange(m + 1, dtype=torch.int64, device=gpu) * k
    dev = nat.step_csr(K, T(pos), T(nrm), T(ev), T(ci), off, T(nbr.reshape(-1)), d, alpha).cpu().numpy()
    # the global delta of flat / new (Denoiser.py:106-107, 138) as the device reduced it
    delta = 0.0
    if kind in ("flat", "new"):
        rows = pos[nbr.reshape(-1)]
        c = (rows.astype(np.float64).mean(0)).astype(np.float32)
        delta = float(np.sqrt(((rows - c) ** 2).sum(1)).max())
    host = nat.host_step_csr(K, pos, nrm, ev, ci, nbr, d, alpha, delta)
    same = (dev.view(np.uint32) == host.view(np.uint32)).all(1)
    if kind in ("flat", "new"):      # (the device's delta comes from its own f32 max; compare to rounding)
        np.testing.assert_allclose(dev, host, rtol=0, atol=1e-6)
    else:
        assert same.all(), f"{kind}: {(~same).sum()} of {m} rows differ; max {np.abs(dev - host).max():.3g}"
