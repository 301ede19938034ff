"""Golden vectors for the batched 3x3 symmetric eigen-decomposition: torch.linalg.eigh on CPU float32 -- the
reference's own call in getBetterFilteredNVT / getNormalFilteredNVT / getNormalFilteredPVT / getPVTDecompositionWithKNN
(Decompositionor.py:211, 276, 300; GraphBuilder.py:111) -- as MKL 2024.2's ssyevd computes it on the CPU of the
container this ran in (AVX-512 path).  MKL takes other code paths on other CPUs, so the tests compare the library's
restatement (pcd_device.h eigh3, through pcd_host_eigh3) with these saved outputs instead of live torch calls.

    python tests/golden/make_eigh_golden.py        -> tests/golden/eigh.npz

Families: random symmetric; rank-1 outer products (a single voting neighbour: the null-space basis is set by
rounding); NVT-like means of unit-normal outer products around 1-3 directions (0 to 0.3 rad of jitter, exact
clusters included); PCA-like 12-point covariances at point spacings 1 .. 1e-6 (ssteqr's block scaling below 2^-15);
matrices scaled across ssyevd's and ssteqr's scaling bounds (1e-37 .. 1e18); exactly repeated eigenvalues.
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def families(rng, m):
    out = {}
    R = rng.normal(size=(m, 3, 3))
    A = ((R + R.transpose(0, 2, 1)) / 2).astype(np.float32)
    out["random"] = A
    n = rng.normal(size=(m, 3))
    n = (n / np.linalg.norm(n, axis=1, keepdims=True)).astype(np.float32)
    out["rank1"] = n[:, :, None] * n[:, None, :]
    T = np.empty((m, 3, 3), np.float32)
    for r in range(m):
        c = rng.integers(1, 33)
        kd = rng.integers(1, 4)
        dirs = rng.normal(size=(kd, 3))
        jit = 0.0 if rng.random() < 0.2 else 10 ** rng.uniform(-7, -0.5)
        nn = dirs[rng.integers(0, kd, c)] + jit * rng.normal(size=(c, 3))
        nn = (nn / np.linalg.norm(nn, axis=1, keepdims=True)).astype(np.float32)
        T[r] = (nn[:, :, None] * nn[:, None, :]).sum(0) / np.float32(c)
    out["nvt"] = T
    for sc in (1.0, 1e-2, 1e-4, 1e-6):
        P = rng.normal(size=(m, 12, 3)) * np.array([1, 1, 0.05]) * sc
        Q = np.linalg.qr(rng.normal(size=(m, 3, 3)))[0]
        P = np.einsum("mij,mkj->mki", Q, P).astype(np.float32)
        c = P - P.mean(1, keepdims=True)
        out[f"pca{sc:g}"] = np.einsum("mki,mkj->mij", c, c).astype(np.float32)
    An = A / np.abs(A).max((1, 2), keepdims=True)
    for sc in (1e-37, 1e-20, 3.0517578125e-05, 3e-5, 3.2e18, 1e18):
        out[f"scaled{sc:g}"] = (An * np.float32(sc)).astype(np.float32)
    D = np.zeros((m, 3, 3), np.float32)
    D[:, 0, 0] = rng.normal(size=m)
    D[:, 1, 1] = D[:, 0, 0]
    D[:, 2, 2] = rng.normal(size=m)
    ax = np.eye(3, dtype=np.float32)[rng.integers(0, 3, (m, 4))]
    out["repeated"] = np.concatenate([D, (ax[..., :, None] * ax[..., None, :]).mean(1), np.zeros((8, 3, 3), np.float32)])
    return out


def main():
    torch.set_num_threads(1)
    rng = np.random.default_rng(21)
    res = {}
    for name, T in families(rng, 1500).items():
        w, v = torch.linalg.eigh(torch.from_numpy(np.ascontiguousarray(T)))
        res[f"{name}_T"] = T
        res[f"{name}_w"] = w.numpy()
        res[f"{name}_v"] = v.numpy()
    res["mkl"] = np.array(torch.__config__.show())
    np.savez_compressed(os.path.join(HERE, "eigh.npz"), **res)
    print("eigh.npz:", ", ".join(k[:-2] for k in res if k.endswith("_T")))


if __name__ == "__main__":
    main()
