"""CPU checks of the C-ABI boundary (include/pcd.h <-> libpcd.so <-> pcd_native), no GPU compute.

* the library loads and exports every entry point the header declares; pcd_native binds exactly those
* argument validation fails with PCD_ERR_ARG + pcd_last_error() before touching a device
* the host builds of the kernels' per-point math (pcd_host_*) agree with the reference's own libraries:
  eigen-decomposition vs MKL torch.linalg.eigh (values AND eigenvector signs), VU smoothing and 3x3 solves vs the
  oracle, MST orientation (host C++) vs the oracle.
"""
import ctypes
import math
import os
import re

import numpy as np
import pytest
import torch

import pcd_native as nat
from oracle import pcd_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pcd.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pcd_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = nat.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), f"libpcd.so does not export {s}"


def test_binding_covers_header_exactly():
    assert sorted(nat.exported_symbols()) == header_symbols()


def test_version_and_limits():
    L = nat.lib()
    assert L.pcd_version() >= 1
    assert L.pcd_max_k() == 64


def test_argument_errors_are_reported():
    L = nat.lib()
    idx = ctypes.c_void_p()
    rc = L.pcd_knn(None, None, 10, 8, None, 64, 0, 0, None, None)
    assert rc == nat.PCD_ERR_ARG
    assert b"grid is null" in L.pcd_last_error()
    rc = L.pcd_grid_build(None, 0, 16, 0.0, None, None, ctypes.byref(idx))
    assert rc == nat.PCD_ERR_ARG and not idx.value
    with pytest.raises(ValueError):
        nat.check(L.pcd_step_csr(99, None, None, None, 0, None, None, None, 0, 1.0, 1.0, None, None), "step")
    with pytest.raises(ValueError):
        nat.check(L.pcd_denoiser_create(None, 16, ctypes.byref(idx)), "create")


def _nvt_tensors(golden):
    f = golden("fandisk_k32")
    pos, n, idx = f["pos0"], f["n0"], f["knn32"]
    vj, nj = pos[idx], n[idx]
    dv = vj - pos[:, None]
    dn = dv / np.maximum(np.linalg.norm(dv, axis=-1, keepdims=True), 1e-12)
    w = (np.arccos(np.abs(np.clip((dn * nj).sum(-1), -1, 1))) > np.float32(math.pi * 5 / 12)).astype(np.float32)
    w[w.sum(1) == 0] = 1
    T = (w[..., None, None] * nj[..., :, None] * nj[..., None, :]).sum(1) / w.sum(1)[:, None, None]
    return T.astype(np.float32)


def _t6(T):
    return np.stack([T[:, 0, 0], T[:, 1, 0], T[:, 2, 0], T[:, 1, 1], T[:, 2, 1], T[:, 2, 2]], 1)


def _eigh_families(golden):
    g = golden("eigh")
    return g, sorted(k[:-2] for k in g.files if k.endswith("_T"))


def test_host_eigh_matches_mkl_bitwise(golden):
    """eigh3 (pcd_device.h: ssyevd = ssytd2 + ssteqr('I') + sormtr with MKL's fma placement, ssyevd's and ssteqr's
    scaling) against torch.linalg.eigh -- the reference's own call -- BIT FOR BIT: eigenvalues and every eigenvector
    component, on every family of tests/golden/eigh.npz (MKL 2024.2's outputs saved by make_eigh_golden.py: random,
    rank-1 single-voter tensors whose null-space basis is set by rounding, NVT-like, PCA covariances down to 1e-6
    spacing, matrices across the scaling bounds, repeated eigenvalues)."""
    g, fams = _eigh_families(golden)
    assert len(fams) >= 14
    for fam in fams:
        w, v = nat.host_eigh3(_t6(g[f"{fam}_T"]))
        np.testing.assert_array_equal(w, g[f"{fam}_w"], err_msg=fam)
        np.testing.assert_array_equal(v, g[f"{fam}_v"], err_msg=fam)


@pytest.mark.parametrize("which", ["nvt", "pca"])
def test_host_eigh_matches_reference_fixtures_bitwise(golden, which):
    """The same restatement on the tensors of the reference's own runs: NVT1 of fandisk at k = 32
    (Decompositionor.py:278-300, the fixture's eigval1 / eigvec1) and the unoriented PCA normals
    (GraphBuilder.py:99-111, steps.npz pca_n = eigvec[..., 0])."""
    if which == "nvt":
        f = golden("fandisk_k32")
        w, v = nat.host_eigh3(_t6(_nvt_tensors(golden)))
        np.testing.assert_array_equal(w, f["eigval1"])
        np.testing.assert_array_equal(v, f["eigvec1"])
    else:
        s = golden("steps")
        vj = torch.from_numpy(s["pos"])[torch.from_numpy(s["knn12_noself"].astype(np.int64))]
        d = vj - vj.mean(dim=1)[:, None]                 # GraphBuilder.py:107-109 evaluated as written
        T = (d[:, :, None] * d[..., None]).sum(dim=1).numpy()
        _, v = nat.host_eigh3(_t6(T))
        np.testing.assert_array_equal(v[..., 0], s["pca_n"])


def test_host_vu_smooth_matches_reference_bitwise(golden):
    """Decomposition.getVUSmoothedNormals (Decompositionor.py:92-106) on the reference's own eigen-decompositions:
    bit-identical (Eᵀ·M·E in torch's summation order, Tensor.norm's fma accumulation)."""
    s = golden("steps")
    for rho in ("a5pi12", "api3"):
        for k in (8, 16):
            ev, evec, n1 = s[f"nvt_{rho}_k{k}_eigval"], s[f"nvt_{rho}_k{k}_eigvec"], s["n1"]
            np.testing.assert_array_equal(nat.host_vu_smooth(ev, evec, n1), s[f"nvt_{rho}_k{k}_vu"], err_msg=(rho, k))


@pytest.mark.parametrize("k", [8, 16])
def test_host_nvt1_chain_matches_reference_bitwise(golden, k):
    """The fused kernels' NVT1 (vote + list-order tensor sums, eigh3, VU smoothing) on the host against the
    reference's getBetterFilteredNVT + getVUSmoothedNormals outputs (steps.npz): every eigenvalue, eigenvector and
    smoothed normal bit-identical, single-voter neighbourhoods included."""
    s = golden("steps")
    pos, n1 = s["pos"], s["n1"]
    knn = s[f"knn{k}"].astype(np.int64)
    m = len(knn)
    for rho_name, rho in (("a5pi12", math.pi * 5 / 12), ("api3", math.pi / 3)):
        t6 = nat.host_nvt_tensor(pos, n1, np.arange(m), np.arange(m + 1) * k, knn.reshape(-1), rho)
        w, v = nat.host_eigh3(t6)
        np.testing.assert_array_equal(w, s[f"nvt_{rho_name}_k{k}_eigval"])
        np.testing.assert_array_equal(v, s[f"nvt_{rho_name}_k{k}_eigvec"])
        np.testing.assert_array_equal(nat.host_vu_smooth(w, v, n1), s[f"nvt_{rho_name}_k{k}_vu"])


def test_host_solve3():
    rng = np.random.default_rng(3)
    A = rng.standard_normal((2000, 3, 3)).astype(np.float32)
    b = rng.standard_normal((2000, 3)).astype(np.float32)
    A[:10, 2] = 0.0                              # exactly singular rows
    A[10:20, :, 0] = 0.0                         # exactly singular column
    x, ok = nat.host_solve3(A, b)
    _, ok_ref = O.inv_ex(A)
    assert (ok == ok_ref).all()
    good = ok & (np.linalg.cond(A.astype(np.float64)) < 1e3)
    xr = np.linalg.solve(A[good].astype(np.float64), b[good].astype(np.float64)[..., None])[..., 0]
    np.testing.assert_allclose(x[good], xr, rtol=1e-4, atol=1e-4)


def test_host_inv3_matches_torch_bitwise(golden):
    """inv3_ref (pcd_device.h, what every position step runs) against torch.linalg.inv_ex -- the reference's own call
    (Denoiser.py:43, 80, 163, 210) -- bit for bit, with the same info mask: torch's outputs saved by
    tests/golden/make_inv_golden.py (torch restates inv_ex as getrf(Aᵀ) + getrs('T', I) through MKL, whose code path
    depends on the CPU, so the reference values are data, not a live call)."""
    g = golden("inv_ex")
    inv, ok = nat.host_inv3(g["A"])
    ok_ref = g["info"] == 0
    assert (ok == ok_ref).all()
    assert ok.mean() > 0.99
    same = (inv.view(np.uint32) == g["inv"].view(np.uint32)).all(axis=(1, 2))
    assert same[ok].all(), f"{(~same[ok]).sum()} of {ok.sum()} inverses differ"


def test_host_solve3_is_inverse_then_product(golden):
    """solve3 = einsum("nij,nj->ni", inv_ex(A), b) as torch computes it (row sums (a0 b0 + a1 b1) + a2 b2), against
    torch's saved outputs."""
    g = golden("inv_ex")
    x, ok = nat.host_solve3(g["A"], g["b"])
    assert (ok == (g["info"] == 0)).all()
    np.testing.assert_array_equal(x[ok], g["x"][ok])


def test_orientation_host_matches_oracle(golden):
    lat = golden("lattice")
    pos = lat["n17_j1_pos"]
    nbr = O.knn_graph_noself(pos, 12)
    n0 = O.pca_normals_unoriented(pos, nbr).astype(np.float32)
    ref = O.orient_normals_mst(pos, n0.copy(), nbr)
    n = torch.from_numpy(n0.copy())
    a = torch.from_numpy(np.repeat(np.arange(len(pos)), 12))
    b = torch.from_numpy(nbr.reshape(-1).copy())
    nat.orient_normals_mst(torch.from_numpy(pos.copy()), n, a, b)
    assert ((n.numpy() * ref).sum(1) > 0.999).mean() > 0.995
    # and with the reference's own oriented normals
    assert (np.sign((n.numpy() * lat["n17_j1_n"]).sum(1)) > 0).mean() > 0.99


def _nvt_pairs(rng, m, k, rho):
    """Rows of k (v_j, n_j) around v_i = 0 whose |c| sits at cos(rho) within 1e-8 .. 1e-4, plus random, parallel
    (no vote in the row) and degenerate (|dv| tiny or zero) pairs."""
    u = rng.standard_normal((m, k, 3)); u /= np.linalg.norm(u, axis=-1, keepdims=True)
    p = rng.standard_normal((m, k, 3)); p -= (p * u).sum(-1, keepdims=True) * u
    p /= np.linalg.norm(p, axis=-1, keepdims=True)
    ct = math.cos(rho)
    rel = rng.choice([-1e-4, -1e-5, -1e-6, -1e-7, -1e-8, 0.0, 1e-8, 1e-7, 1e-6, 1e-5, 1e-4], size=(m, k))
    a = ct * (1 + rel) * rng.choice([-1.0, 1.0], size=(m, k))
    scale = rng.uniform(0.9, 1.1, size=(m, k))
    nj = scale[..., None] * (a[..., None] * u + np.sqrt(np.maximum(1 - a * a, 0))[..., None] * p)
    length = 10.0 ** rng.uniform(-4, 2, size=(m, k))
    dv = u * length[..., None]
    rnd = rng.random((m, k)) < 0.2                                  # random pairs
    nj[rnd] = rng.standard_normal((int(rnd.sum()), 3))
    nj[m // 8:m // 4] = u[m // 8:m // 4] * rng.choice([-1.0, 1.0], size=(m // 4 - m // 8, k, 1))   # no vote
    dv[:, 0] *= np.where(rng.random(m) < 0.1, 1e-13, 1.0)[:, None]   # below F.normalize's eps
    dv[:, 1] *= np.where(rng.random(m) < 0.5, 0.0, 1.0)[:, None]     # zero (the row itself)
    return dv.astype(np.float32), nj.astype(np.float32)


def test_host_nvt_vote_and_sums_match_reference_expression():
    """The fused kernels' squared-form vote with its exact fallback decides every pair exactly like the reference's
    acos(|clamp(normalize(dv) . n_j)|) > rho in f32 (same libm acosf), and the tensor sums (voting rows in list
    order, all-ones fallback) are bit-identical to a sequential f32 restatement (Decompositionor.py:278-300)."""
    libm = ctypes.CDLL("libm.so.6")
    libm.acosf.restype = ctypes.c_float
    libm.acosf.argtypes = [ctypes.c_float]
    acosf = np.vectorize(lambda x: libm.acosf(float(x)), otypes=[np.float32])
    rng = np.random.default_rng(17)
    m, k = 2048, 32
    F = np.float32
    for rho in (math.pi * 5 / 12, 0.3, math.pi / 2 + 0.01):
        dv, nj = _nvt_pairs(rng, m, k, rho)
        # rows 0..7: |c| at the f32 neighbours of cos(rho) (dv along an axis with power-of-two length, so the
        # reference's normalisation is exact and c is exactly the chosen value)
        ct = np.float32(math.cos(np.float32(rho)))
        cs = np.array([ct + i * np.spacing(ct) for i in range(-128, 128)], F)[:8 * k]
        for r in range(8):
            axis = r % 3
            L = F(2.0 ** (r - 3))
            sel = cs[r * k:(r + 1) * k]
            dv[r] = 0
            dv[r, :, axis] = L * (1 if r % 2 == 0 else -1)
            nj[r] = 0
            nj[r, :, axis] = sel * (1 if r < 4 else -1)
            nj[r, :, (axis + 1) % 3] = np.sqrt(np.maximum(1 - sel.astype(np.float64) ** 2, 0)).astype(F)
        # layout: point 0 = the centre at the origin, pairs after it
        pos = np.concatenate([np.zeros((1, 3), F), dv.reshape(-1, 3)])
        n = np.concatenate([np.zeros((1, 3), F), nj.reshape(-1, 3)])
        ci = np.zeros(m, np.int64)
        off = np.arange(m + 1, dtype=np.int64) * k
        nbr = 1 + np.arange(m * k, dtype=np.int64)
        T = nat.host_nvt_tensor(pos, n, ci, off, nbr, rho)
        d = pos[nbr].reshape(m, k, 3) - pos[0]
        den = np.maximum(np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]), F(1e-12))
        dn = d / den[..., None]
        c = np.abs(np.clip((dn[..., 0] * nj[..., 0] + dn[..., 1] * nj[..., 1]) + dn[..., 2] * nj[..., 2], -1, 1))
        w = acosf(c) > F(rho)
        w[w.sum(1) == 0] = True
        acc = np.zeros((m, 6), F)
        comps = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
        for t in range(k):
            for q, (x, y) in enumerate(comps):
                acc[:, q] = np.where(w[:, t], acc[:, q] + nj[:, t, x] * nj[:, t, y], acc[:, q]).astype(F)
        ref = acc / w.sum(1).astype(F)[:, None]
        np.testing.assert_array_equal(T, ref)
