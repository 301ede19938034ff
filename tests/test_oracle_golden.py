"""Pin the CPU oracle (oracle/pcd_oracle.py) against golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py).  CPU only; these establish that the checker used by the GPU parity tests is right.

Tolerances follow SURVEY.md §8(c): discrete decisions (kNN sets, w_ij thresholds, classes, clamps) must agree except
on near-ties; continuous outputs agree to fp32 rounding.
"""
import math

import numpy as np
import pytest

from oracle import pcd_oracle as O


def angle(a, b):
    """Unsigned angle between line directions, accurate near 0 (float64 chord, not arccos of an fp32 dot)."""
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    a = a / np.linalg.norm(a, axis=-1, keepdims=True)
    b = b / np.linalg.norm(b, axis=-1, keepdims=True)
    s = np.sign((a * b).sum(-1, keepdims=True)); s[s == 0] = 1
    return 2 * np.arcsin(np.clip(np.linalg.norm(a - s * b, axis=-1) / 2, 0, 1))


@pytest.fixture(scope="module")
def fan(golden):
    return golden("fandisk_k32")


def test_knn_frozen_snapshot_matches_reference(fan):
    knn = O.FrozenKNN(fan["pos0"])
    idx, d = knn.query(fan["pos0"], 32)
    assert (idx == fan["knn32"]).mean() > 0.9999
    np.testing.assert_allclose(d, fan["knn32_d"], rtol=0, atol=1e-12)


def test_mean_edge_length_and_d(fan):
    knn = O.FrozenKNN(fan["pos0"])
    l = O.mean_edge_length(fan["pos0"], knn)
    assert abs(l - float(fan["l"])) < 1e-6 * float(fan["l"])


def test_oracle_eigh_is_mkls_bitwise(golden):
    """oracle/eigh3_mkl.c (LAPACK ssyevd's loops with MKL 2024.2's AVX-512 fma placement) against torch.linalg.eigh's
    saved outputs (tests/golden/eigh.npz: random, rank-1 single-voter, NVT-like, PCA covariances down to 1e-6
    spacing, matrices across ssyevd's and ssteqr's scaling bounds, repeated eigenvalues): every eigenvalue and every
    eigenvector component bit for bit, so the oracle does not depend on the host's MKL code path."""
    g = golden("eigh")
    fams = sorted(k[:-2] for k in g.files if k.endswith("_T"))
    assert len(fams) >= 14
    for fam in fams:
        w, v = O.eigh(g[f"{fam}_T"])
        np.testing.assert_array_equal(w, g[f"{fam}_w"], err_msg=fam)
        np.testing.assert_array_equal(v, g[f"{fam}_v"], err_msg=fam)


def test_oracle_norm3_is_torchs():
    """Tensor.norm(dim=1) / F.normalize on CPU float32 accumulate the squares with fmas: norm3 restates it."""
    import torch
    rng = np.random.default_rng(3)
    x = (rng.normal(size=(50_000, 3)) * rng.uniform(1e-3, 1e3, size=(50_000, 1))).astype(np.float32)
    np.testing.assert_array_equal(O.norm3(x), torch.from_numpy(x).norm(dim=1).numpy())


@pytest.mark.parametrize("k", [32, 16])
def test_nvt1_matches_reference_bitwise(golden, k):
    """NVT1 of one Processor.denoise loop body (getBetterFilteredNVT + getVUSmoothedNormals, Decompositionor.py:92-106,
    278-300) on fandisk at k = 32 and at Processor.denoise()'s default k = 16: eigenvalues, eigenvectors and the
    smoothed normals f_n bit-identical to the reference's run."""
    fan = golden(f"fandisk_k{k}")
    ci = np.arange(len(fan["pos0"]))
    w, v = O.better_filtered_nvt(fan["pos0"], fan["n0"], ci, fan[f"knn{k}"], math.pi * 5 / 12)
    np.testing.assert_array_equal(w, fan["eigval1"])
    np.testing.assert_array_equal(v, fan["eigvec1"])
    np.testing.assert_array_equal(O.vu_smoothed_normals(w, v, fan["n0"]), fan["it1_f_n"])


@pytest.mark.parametrize("k", [32, 16])
def test_iteration1_stages(golden, k):
    """One Processor.denoise loop body at k = 32 and at its default k = 16 (Processor.py:119-139): classes, f_n and
    NVT2's eigenvalues bit-identical to the reference's; positions after each Gauss-Seidel phase within 5e-7 x bbox
    (the flat step's exp() and global centre are the only operations not restated to the bit: torch's vectorised
    exp and its float32 mean; measured max 1.8e-7, ~90 % of the rows exact)."""
    fan = golden(f"fandisk_k{k}")
    knn = O.FrozenKNN(fan["pos0"])
    rec = {}
    pos, f_n, cls = O.denoise_iteration(fan["pos0"], fan["n0"], knn, float(fan["d"]), k, 8, record=rec)
    np.testing.assert_array_equal(cls, fan["it1_classes"])
    np.testing.assert_array_equal(f_n, fan["it1_f_n"])
    np.testing.assert_array_equal(rec["eigval2"], fan["it1_eigval2"])
    bbox = np.linalg.norm(fan["pos0"].max(0) - fan["pos0"].min(0))
    for key in range(3):
        dev = np.linalg.norm(rec[f"pos_after_{key}"] - fan[f"it1_pos_after_{key}"], axis=1) / bbox
        assert (dev == 0).mean() > 0.85 and np.percentile(dev, 99.9) < 1e-7 and dev.max() < 5e-7, \
            (key, (dev == 0).mean(), np.percentile(dev, 99.9), dev.max())


def test_ten_iterations_within_fp32_fp64_envelope(fan):
    """End-to-end: the oracle's CD trajectory stays within the reference's own fp32-vs-fp64 spread."""
    knn = O.FrozenKNN(fan["pos0"])
    pos, n = fan["pos0"].copy(), fan["n0"].copy()
    cds = [O.chamfer(fan["gt"], pos).mean()]
    for _ in range(10):
        pos, n, _ = O.denoise_iteration(pos, n, knn, float(fan["d"]), 32, 8)
        cds.append(O.chamfer(fan["gt"], pos).mean())
    ref32, ref64 = fan["cd_f32"], fan["cd_f64"]
    env = np.maximum(np.abs(ref32 - ref64), 0.02 * ref32)
    assert np.all(np.abs(np.asarray(cds) - ref32) <= 2 * env + 1e-6), (cds, ref32, ref64)
    assert abs(cds[1] - ref32[1]) / ref32[1] < 1e-3


def test_processor_denoise_verbatim(golden):
    g = golden("fandisk_denoise")
    pos, n = O.denoise(g["pos0"], g["n0"], iterations=2, k=16, k_update=8)
    bbox = np.linalg.norm(g["pos0"].max(0) - g["pos0"].min(0))
    dev = np.linalg.norm(pos - g["pos"], axis=1) / bbox
    assert np.percentile(dev, 99) < 5e-3
    assert np.median(dev) < 1e-5


@pytest.fixture(scope="module")
def steps(golden):
    return golden("steps")


@pytest.mark.parametrize("rho", ["a5pi12", "api3"])
@pytest.mark.parametrize("k", [8, 16])
def test_nvt_vu_classes(steps, rho, k):
    pos, n1 = steps["pos"], steps["n1"]
    ci = np.arange(len(pos))
    r = math.pi * 5 / 12 if rho == "a5pi12" else math.pi / 3
    w, v = O.better_filtered_nvt(pos, n1, ci, steps[f"knn{k}"], r)
    # the whole NVT1 chain -- vote, list-order tensor sums, MKL-exact eigh, VU smoothing -- bit for bit
    np.testing.assert_array_equal(w, steps[f"nvt_{rho}_k{k}_eigval"])
    np.testing.assert_array_equal(v, steps[f"nvt_{rho}_k{k}_eigvec"])
    vu = O.vu_smoothed_normals(w, v, n1)
    np.testing.assert_array_equal(vu, steps[f"nvt_{rho}_k{k}_vu"])
    cls = O.classes(steps[f"nvt_{rho}_k{k}_eigval"])
    assert (cls == steps[f"nvt_{rho}_k{k}_classes"]).all()
    feats = np.stack(O.nvt_features(steps[f"nvt_{rho}_k{k}_eigval"]), 1)
    np.testing.assert_allclose(feats, steps[f"nvt_{rho}_k{k}_features"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("alpha", [1.0, 0.2])
@pytest.mark.parametrize("kind", ["flat", "edge", "feature", "corner", "new"])
def test_denoiser_steps(steps, kind, alpha):
    pos, n1, sub = steps["pos"], steps["n1"], steps["subset"]
    nbr = steps["knn8"][sub]
    d = float(steps["d"])
    tag = f"a{alpha}"
    bbox = np.linalg.norm(pos.max(0) - pos.min(0))
    for dd, suffix in ((d, ""), (1e9, "_noclamp")):
        key = f"{kind}_{tag}{suffix}"
        if key not in steps:
            continue
        if kind == "edge":
            out = O.edge_step(pos, n1, steps["edge_vectors"], sub, nbr, dd, alpha)
        else:
            out = O.STEPS[kind](pos, n1, sub, nbr, dd, alpha)
        dev = np.linalg.norm(out - steps[key], axis=1) / bbox
        if kind in ("edge", "feature", "corner"):
            # the solve steps are restated op for op (torch's inv_ex and einsum, the same sums in list order): the
            # reference's own output bit for bit
            np.testing.assert_array_equal(out, steps[key], err_msg=key)
            continue
        # flat / new: the global centre is an f64 mean here, a float32 torch mean (cascade summation) there
        assert np.percentile(dev, 99.9) < 1e-5, (key, np.percentile(dev, 99.9))
        assert dev.max() < 1e-5, (key, dev.max())


def test_dummy_step(steps):
    sub = steps["subset"]
    np.testing.assert_array_equal(steps["dummy_a1.0"], steps["pos"][sub])


def test_pca_normals_up_to_sign(steps):
    nbr = O.knn_graph_noself(steps["pos"], 12)
    assert (np.sort(nbr, 1) == np.sort(steps["knn12_noself"], 1)).mean() > 0.999
    n = O.pca_normals_unoriented(steps["pos"], steps["knn12_noself"])
    np.testing.assert_array_equal(n, steps["pca_n"])          # torch's reduction order + the MKL-exact eigh


def test_lattice_kat(golden):
    lat = golden("lattice")
    for tag in ("n9_j0", "n17_j0", "n9_j1", "n17_j1"):
        pos, n = lat[f"{tag}_pos"], lat[f"{tag}_n"]
        knn = O.FrozenKNN(pos)
        (w2, _), f_n, _ = O.feature_decomposition(pos, n, knn, 16)
        cls = O.classes(w2)
        acc = (cls == lat[f"{tag}_gt"]).mean()
        # exact lattices are full of kNN distance ties; scipy's tie order is implementation-defined
        assert abs(acc - float(lat[f"{tag}_acc"])) < 0.01, (tag, acc, float(lat[f"{tag}_acc"]))
        if tag.endswith("j1"):
            assert (cls == lat[f"{tag}_classes"]).mean() > 0.995


def test_orientation_mst(golden):
    lat = golden("lattice")
    pos = lat["n9_j1_pos"]
    nbr = O.knn_graph_noself(pos, 12)
    n = O.pca_normals_unoriented(pos, nbr)
    n = O.orient_normals_mst(pos, n, nbr)
    agree = np.abs((n * lat["n9_j1_n"]).sum(1))
    signs = np.sign((n * lat["n9_j1_n"]).sum(1))
    assert np.percentile(agree, 1) > 0.99
    assert (signs > 0).mean() > 0.99


def test_mesh_update(golden):
    m = golden("mesh_update")
    v1 = O.mesh_update(m["v"], m["f"], m["n"], k=1)
    np.testing.assert_allclose(v1, m["v_k1"], rtol=0, atol=1e-12)
    v15 = O.mesh_update(m["v"], m["f"], m["n"], k=15)
    np.testing.assert_allclose(v15, m["v_k15"], rtol=0, atol=1e-10)


def test_metrics(golden):
    m = golden("metrics")
    np.testing.assert_allclose(O.chamfer(m["a"], m["b"]), m["chamfer"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(O.paper_distance(m["a"], m["b"]), m["paper"], rtol=1e-5, atol=1e-9)


# ------------------------------------------------------------------ CPSD path
@pytest.fixture(scope="module")
def cpsd(golden):
    return golden("cpsd")


@pytest.mark.parametrize("tag", ["r1", "r2"])
def test_radius_selection_matches_reference(cpsd, tag):
    slices, j = O.radius_selection(cpsd["pos"], cpsd["pos"], float(cpsd[f"sel_{tag}_radius"]))
    np.testing.assert_array_equal(slices, cpsd[f"sel_{tag}_slices"])
    np.testing.assert_array_equal(j, cpsd[f"sel_{tag}_j"])


def test_martin_feature_decomposition_matches_reference(cpsd):
    pos, n, d = cpsd["pos"], cpsd["n"], float(cpsd["d"])
    slices, j = O.radius_selection(pos, pos, d)
    ci = np.arange(len(pos))
    w1, v1 = O.normal_filtered_nvt(n, ci, slices, j, 0.9)
    np.testing.assert_array_equal(w1, cpsd["nvt_eigval"])
    np.testing.assert_array_equal(v1, cpsd["nvt_eigvec"])
    w2, v2, fn = O.martin_feature_decomposition(pos, pos, n, d, 0.9)
    np.testing.assert_array_equal(fn, cpsd["f_n"])
    np.testing.assert_array_equal(w2, cpsd["pvt_eigval"])
    np.testing.assert_array_equal(v2, cpsd["pvt_eigvec"])
    np.testing.assert_array_equal(O.vu_features(w2, 0.3), cpsd["vu_classes"])


def angle64(a, b):
    """Angle between row vectors in float64 (arccos of an f32 dot cannot resolve below ~5e-4 rad)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.arctan2(np.linalg.norm(np.cross(a, b), axis=1), (a * b).sum(1))


def test_cpsd_driver_oracle_matches_reference(golden):
    """pcd_oracle.cpsd_iteration (the CPSD driver's loop body, PostProcessing.ipynb:1041-1062) against the reference's
    own run of that loop on fandisk (cpsd.npz drv_*): iteration 1 at the single-iteration gates (median exact, p99
    1e-5 x bbox), iteration 2 within the chaotic envelope of SURVEY §8(c)."""
    c = golden("cpsd")
    pos0, n0, d = c["pos"], c["n"], float(c["drv_d"])
    bbox = float(np.linalg.norm(pos0.max(0) - pos0.min(0)))
    knn = O.FrozenKNN(pos0)
    rp, rn = pos0.copy(), n0.copy()
    for it in (1, 2):
        rp, rn = O.cpsd_iteration(pos0, rp, rn, pos0, knn, d)
        dev = np.linalg.norm(rp - c[f"drv_pos_it{it}"], axis=1) / bbox
        np.testing.assert_array_equal(rn, c[f"drv_n_it{it}"])   # f_n: the radius NVT + VU chain, bit for bit
        if it == 1:
            # only the flat step's exp() and global centre are not restated to the bit (measured: 99.4 % of the rows
            # exact, max 5.7e-9 x bbox)
            assert np.median(dev) == 0 and np.percentile(dev, 99) <= 1e-8 and dev.max() < 1e-7, dev.max()
        else:
            assert np.median(dev) < 1e-5 and np.percentile(dev, 99) < 5e-3, np.percentile(dev, 99)


def test_oracle_inv_ex_is_torchs_bitwise(golden):
    """The oracle's numpy restatements of torch.linalg.inv_ex (getrf(A^T) + getrs('T') in MKL's AVX-512 arithmetic) and
    of torch's CPU einsum are torch's own results bit for bit: saved torch outputs (tests/golden/make_inv_golden.py,
    random, SPD-like and singular 3x3 systems), so the check does not depend on this host's MKL code path."""
    g = golden("inv_ex")
    inv, ok = O.inv_ex(g["A"])
    assert (ok == (g["info"] == 0)).all()
    np.testing.assert_array_equal(inv[ok], g["inv"][ok])
    x = O._einsum("nij,nj->ni", g["inv"], g["b"])
    np.testing.assert_array_equal(x, g["x"])
    np.testing.assert_array_equal(O._einsum("nkij,nkj->nki", g["M4"], g["v4"]), g["y4"])
    np.testing.assert_array_equal(O._einsum("nkij,nj->nki", g["M4"], g["v4"][:, 0]), g["y5"])
