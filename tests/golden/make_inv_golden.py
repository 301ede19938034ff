"""Golden vectors for the 3x3 solves of the position steps: torch.linalg.inv_ex (Denoiser.py:43, 80, 163, 210) and
torch.einsum("nij,nj->ni") / ("nkij,nkj->nki") / ("nkij,nj->nki") as torch computes them on the CPU of the container this ran in
(torch 2.10, MKL's getrf(A^T) + getrs('T')).  MKL takes other code paths on other CPUs, so the tests compare the
library's and the oracle's restatements against these saved outputs instead of live torch calls.

    python tests/golden/make_inv_golden.py        -> tests/golden/inv_ex.npz
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def inv_cases(rng, m):
    """SPD systems shaped like feature_step's A (I + n nᵀ + Σ n_j n_jᵀ + k_u n nᵀ), edge_step-like sums of rank-2
    terms, random Gaussian matrices, and exactly singular ones (3m matrices)."""
    u = lambda a: a / np.linalg.norm(a, axis=-1, keepdims=True)
    n = u(rng.normal(size=(m, 3)))
    nj = u(n[:, None, :] + 0.3 * rng.normal(size=(m, 8, 3)))
    feat = np.eye(3)[None] + 9 * n[:, :, None] * n[:, None, :] + (nj[..., :, None] * nj[..., None, :]).sum(1)
    y = u(rng.normal(size=(m, 3)))
    p = nj - (nj * y[:, None]).sum(-1, keepdims=True) * y[:, None]
    edge = (p[..., :, None] * p[..., None, :]).sum(1) + 8 * y[:, :, None] * y[:, None, :]
    gauss = rng.normal(size=(m, 3, 3))
    A = np.concatenate([feat, edge, gauss]).astype(np.float32)
    A[:50, 2] = 0.0                                # exactly singular rows / columns
    A[50:100, :, 1] = 0.0
    A[100:150, 0] = A[100:150, 1]                  # equal rows
    return A


def main():
    torch.set_num_threads(1)
    rng = np.random.default_rng(11)
    A = inv_cases(rng, 4000)
    b = (rng.normal(size=(A.shape[0], 3)) * 10).astype(np.float32)
    M4 = rng.normal(size=(2000, 8, 3, 3)).astype(np.float32)
    v4 = rng.normal(size=(2000, 8, 3)).astype(np.float32)
    inv, info = torch.linalg.inv_ex(torch.from_numpy(A))
    x = torch.einsum("nij,nj->ni", inv, torch.from_numpy(b))
    y4 = torch.einsum("nkij,nkj->nki", torch.from_numpy(M4), torch.from_numpy(v4))
    y5 = torch.einsum("nkij,nj->nki", torch.from_numpy(M4), torch.from_numpy(v4[:, 0]))
    np.savez_compressed(os.path.join(HERE, "inv_ex.npz"), A=A, b=b, inv=inv.numpy(), info=info.numpy(),
                        x=x.numpy(), M4=M4, v4=v4, y4=y4.numpy(), y5=y5.numpy(), torch=torch.__version__)


if __name__ == "__main__":
    main()
