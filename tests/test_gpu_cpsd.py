"""GPU parity of the CPSD ("Martin") feature path: radius selection, normal-filtered NVT / PVT, VU
features, against the reference's golden vectors (tests/golden/cpsd.npz, make_golden.py gen_cpsd) and the oracle.

Tolerances: radius selections identical (same float64 membership test as scipy); the normal-filtered NVT, VU
smoothing, the normal-filtered PVT and the VU classes bit-identical to the reference's (sums in the reference's order,
the MKL-exact eigh); the corner step bit-identical on the reference's inputs; the driver's first iteration median 0,
p99 <= 1e-8 x bbox (the flat step's exp() and float32 global mean are the only operations not restated to the bit).
"""
import math

import numpy as np
import pytest
import torch

from oracle import pcd_oracle as O
from Pointcloud.Modules.Object import Pointcloud
from Pointcloud.Modules.Processor import Processor
from conftest import report

pytestmark = pytest.mark.gpu


def T(x, dev):
    return torch.as_tensor(np.ascontiguousarray(x)).to(dev)


def angle64(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.arctan2(np.linalg.norm(np.cross(a, b), axis=1), (a * b).sum(1))


@pytest.fixture(scope="module")
def cpsd(golden):
    return golden("cpsd")


@pytest.fixture(scope="module")
def proc(cpsd, gpu):
    return Processor(Pointcloud(T(cpsd["pos"], gpu).clone(), T(cpsd["n"], gpu).clone()))


@pytest.mark.parametrize("tag", ["r1", "r2"])
def test_radius_selection_identical_to_reference(cpsd, proc, tag):
    sel = proc.selector.getPointsInRangeSelection(float(cpsd[f"sel_{tag}_radius"]))
    np.testing.assert_array_equal(sel.slices.cpu().numpy(), cpsd[f"sel_{tag}_slices"])
    np.testing.assert_array_equal(sel.j.cpu().numpy(), cpsd[f"sel_{tag}_j"])
    assert sel.j.dtype == torch.int64


def test_radius_selection_subset_and_moved_queries(cpsd, proc, gpu):
    """Vectorized radii over a subset of moved positions (queries against the FROZEN snapshot)."""
    g = torch.Generator().manual_seed(4)
    idx = torch.randperm(len(cpsd["pos"]), generator=g)[:1500].sort().values
    radii = torch.rand(1500, generator=g) * 2 * float(cpsd["d"])
    pos_before = proc.graph.pos.clone()
    proc.graph.pos += 0.05 * torch.randn(proc.graph.pos.shape, generator=g).to(gpu)
    try:
        sel = proc.selector.getPointsInRangeSelectionVectorized(radii.to(gpu), idx.to(gpu))
        tree_pts = cpsd["pos"]
        q = proc.graph.pos[idx.to(gpu)].cpu().numpy()
        tree = O.cKDTree(tree_pts.astype(np.float64))
        lists = tree.query_ball_point(q.astype(np.float64), radii.numpy().astype(np.float64), return_sorted=True)
        ref_j = np.concatenate([np.asarray(x, np.int64) for x in lists])
        ref_s = np.concatenate([[0], np.cumsum([len(x) for x in lists])])
        np.testing.assert_array_equal(sel.slices.cpu().numpy(), ref_s)
        np.testing.assert_array_equal(sel.j.cpu().numpy(), ref_j)
        np.testing.assert_array_equal(sel.i.cpu().numpy(), idx.numpy())
    finally:
        proc.graph.pos.copy_(pos_before)


def test_radius_selection_edge_cases(proc, gpu):
    N = proc.graph.num_nodes
    zero = proc.selector.getPointsInRangeSelectionVectorized(torch.zeros(N, device=gpu))
    lens = zero.slices.diff().cpu().numpy()
    assert lens.min() >= 1                          # radius 0 still holds the point itself (distance 0 <= 0)
    neg = proc.selector.getPointsInRangeSelectionVectorized(torch.full((N,), -1.0, device=gpu))
    assert int(neg.slices[-1]) == 0 and neg.j.numel() == 0
    with pytest.raises(AssertionError):
        proc.selector.getPointsInRangeSelectionVectorized(torch.zeros(N - 1, device=gpu))


def test_martin_feature_decomposition(cpsd, proc):
    dec, fn = proc.getMartinFeatureDecomposition(r=float(cpsd["d"]))
    fn, w, v = fn.cpu().numpy(), dec.eigval.cpu().numpy(), dec.eigvec.cpu().numpy()
    report(f"martin: f_n exact {(fn == cpsd['f_n']).all(1).mean():.6f}, PVT eigval exact "
           f"{(w == cpsd['pvt_eigval']).all(1).mean():.6f}, eigvec exact {(v == cpsd['pvt_eigvec']).all((1, 2)).mean():.6f}")
    np.testing.assert_array_equal(fn, cpsd["f_n"])
    np.testing.assert_array_equal(w, cpsd["pvt_eigval"])
    np.testing.assert_array_equal(v, cpsd["pvt_eigvec"])
    np.testing.assert_array_equal(dec.getVUFeatures(tau=0.3).cpu().numpy(), cpsd["vu_classes"])
    # the PVT kernel alone, fed the GPU's own f_n: the oracle on identical inputs, bit for bit
    pos = cpsd["pos"]
    slices, j = O.radius_selection(pos, pos, float(cpsd["d"]))
    w_ref, v_ref = O.normal_filtered_pvt(pos, fn, np.arange(len(pos)), slices, j, 0.9)
    np.testing.assert_array_equal(w, w_ref)
    np.testing.assert_array_equal(v, v_ref)


def test_normal_filtered_nvt(cpsd, proc):
    sel = proc.selector.getPointsInRangeSelection(float(cpsd["d"]))
    nvt = proc.decompositionor.getNormalFilteredNVT(sel, proc.graph.n, 0.9)
    np.testing.assert_array_equal(nvt.eigval.cpu().numpy(), cpsd["nvt_eigval"])
    np.testing.assert_array_equal(nvt.eigvec.cpu().numpy(), cpsd["nvt_eigvec"])


def test_vu_decomposition(cpsd, proc):
    vu = proc.getVUDecomposition()
    ref = cpsd["vud_eigval"]
    scale = np.abs(ref).max(1, keepdims=True) + 1e-30
    err = np.abs(vu.eigval.cpu().numpy() - ref) / scale
    # the radius is 2 x the mean kNN(6) edge length, an f64 mean here and a float32 torch mean there, so a member
    # at the boundary can differ: reported, gated on the eigenvalues
    report(f"VU decomposition: eigval exact {(err == 0).all(1).mean():.6f}, max rel {err.max():.3g}")
    assert np.percentile(err, 99) < 1e-5 and np.median(err) < 1e-6, np.percentile(err, [50, 99, 100])


def test_pvt_empty_neighbourhood_and_all_rejected(cpsd, gpu):
    """Rows with no neighbours get the cross-product samples; rows where no neighbour votes use every neighbour."""
    pos = cpsd["pos"][:200].astype(np.float32)
    n = cpsd["n"][:200].astype(np.float32)
    n2 = n.copy()
    n2[1::2] *= -1                                   # opposite normals never vote at rho = 0.1
    ci = np.arange(200)
    slices = np.concatenate([[0], np.cumsum(np.where(ci % 5 == 0, 0, 3))]).astype(np.int64)
    seg = np.repeat(ci, np.diff(slices))
    j = ((seg + np.tile([1, 2, 3], 200)[:len(seg)]) % 200).astype(np.int64)
    w_ref, _ = O.normal_filtered_pvt(pos, n2, ci, slices, j, 0.1)
    import pcd_native as nat
    w, _ = nat.pvt_normal_csr(T(pos, gpu), T(n2, gpu), T(ci.astype(np.int64), gpu), T(slices, gpu), T(j, gpu), 0.1)
    scale = np.abs(w_ref).max(1, keepdims=True) + 1e-30
    assert (np.abs(w.cpu().numpy() - w_ref) / scale).max() < 1e-5


def test_cpsd_corner_step(cpsd, proc):
    """The CPSD driver's corner phase (PostProcessing.ipynb:1041-1062) on the reference's classes and f_n."""
    corners = torch.as_tensor(cpsd["corner_idx"], device=proc.graph.pos.device)
    sel8 = proc.selector.getKNNSelection(8)
    out = proc.denoiser.corner_step(sel8.filter(corners), T(cpsd["f_n"], proc.graph.pos.device),
                                    float(cpsd["d"]) * 20000, 1.0).cpu().numpy()
    bbox = np.linalg.norm(cpsd["pos"].max(0) - cpsd["pos"].min(0))
    dev = np.linalg.norm(out - cpsd["corner_pos"], axis=1) / bbox
    report(f"cpsd corner step: exact {(dev == 0).mean():.4f} max {dev.max():.3g} over {len(dev)} corners")
    # inv_ex + einsum restated operation for operation, the sums in list order: the reference's output bit for bit
    np.testing.assert_array_equal(out, cpsd["corner_pos"])


def test_cpsd_driver_matches_reference(cpsd, gpu):
    """The 50-iteration CPSD driver (PostProcessing.ipynb:1041-1062) as Processor.cpsdDenoise: its first two
    iterations against the REFERENCE's own run of the notebook loop on fandisk (make_golden.py gen_cpsd: drv_pos_it1/2,
    d = 2 l as the notebook computes it) -- one iteration within median 1e-6, p99 5e-5 x bbox (its eigen-solves carry
    ~1e-7 relative differences into the steps), the second within the loop's chaotic envelope; the global clamp holds."""
    pos0, n0 = cpsd["pos"], cpsd["n"]
    d = float(cpsd["drv_d"])
    bbox = float(np.linalg.norm(pos0.max(0) - pos0.min(0)))
    for it in (1, 2):
        ref = cpsd[f"drv_pos_it{it}"]
        v = T(pos0, gpu).clone()
        proc = Processor(Pointcloud(v, T(n0, gpu).clone()))
        proc.cpsdDenoise(iterations=it, d=d)                         # original_pos = the call's input, as the ipynb
        dev = np.linalg.norm(v.cpu().numpy() - ref, axis=1) / bbox
        report(f"cpsd driver it{it}: exact {np.mean(dev == 0):.4f} median {np.median(dev):.3g} "
              f"p99 {np.percentile(dev, 99):.3g} max {dev.max():.3g}")
        # n := f_n (radius NVT + VU smoothing): bit-identical to the reference's, iteration after iteration
        np.testing.assert_array_equal(proc.graph.n.cpu().numpy(), cpsd[f"drv_n_it{it}"])
        if it == 1:
            # (round 5, before the MKL-exact eigh: median 4.9e-7, p99 1.8e-5 -- the eigen-solves' last bits); now
            # only the flat step's exp() / global centre differ: measured exact on 99.9 % of the rows, max 1.8e-10
            assert np.median(dev) == 0 and np.percentile(dev, 99) <= 1e-8 and dev.max() <= 1e-6, \
                (np.median(dev), np.percentile(dev, 99), dev.max())
        else:
            assert np.median(dev) == 0 and np.percentile(dev, 99) <= 1e-6, (np.median(dev), np.percentile(dev, 99))
        assert proc.graph.pos is v                                   # updated in place
        moved = np.linalg.norm(v.cpu().numpy() - pos0, axis=1)
        assert moved.max() < d                                        # the global clamp (ipynb:1060-1061)

@pytest.mark.parametrize("rscale", [1.0, "lds32", 1.8, 2.5],
                         ids=["r_d", "r_32_lds_slots", "r_1.8d_global_slots", "r_2.5d_global_slots"])
def test_cpsd_fused_equals_op_by_op(cpsd, gpu, rscale):
    """pcd_cpsd_iterate (the whole loop in one call: radius members sorted in registers / LDS, the fused loop's Jacobi
    phases with the global clamp) against the same operators run op by op through the drop-in classes
    (cpsdDenoise(fused=False)): 2 iterations within 1e-6 x bbox (the flat step's global centre is reduced in two
    different orders).  The call starts with 16 member slots (k_cpsd_nvt<16>, LDS only).  "lds32" picks the first
    radius in 1.0-1.25 d whose largest selection holds 17-32 members (asserted): the first pass overflows and the
    replay runs with 32 slots, all of them in LDS (kCpsdLdsSlots = 32, k_cpsd_nvt<32>).  At r = 1.8 d (~50 members) and 2.5 d (~100, at most ~190) the slots
    grow past the 32 LDS slots into the row's own column of the member-row buffer -- the result must depend on none
    of it."""
    pos0, n0 = cpsd["pos"], cpsd["n"]
    d = float(cpsd["drv_d"])
    bbox = float(np.linalg.norm(pos0.max(0) - pos0.min(0)))
    if rscale == "lds32":          # the LDS-only 32-slot path: the largest selection between 17 and 32 members
        sel = Processor(Pointcloud(T(pos0, gpu).clone())).selector
        top = {x: int(sel.getPointsInRangeSelection(d * x).slices.diff().max()) for x in (1.0, 1.05, 1.1, 1.15, 1.2, 1.25)}
        fits = [x for x, m in top.items() if 16 < m <= 32]
        assert fits, top
        rscale = fits[0]
    out = {}
    for fused in (True, False):
        proc = Processor(Pointcloud(T(pos0, gpu).clone(), T(n0, gpu).clone()))
        if rscale != 1.0:          # a wider selection than the driver's r = d (the global clamp stays d)
            proc.getMartinFeatureDecomposition = (lambda f: (lambda r, rho=0.9: f(r * rscale, rho)))(
                proc.getMartinFeatureDecomposition)
        if fused:
            import pcd_native as nat
            dn = proc._fused_for(8)
            dn.load(proc.graph.pos, proc.graph.n)
            dn.cpsd_iterate(nat.make_cpsd_params(r=d * rscale, d=d), 2)
            p = torch.empty_like(proc.graph.pos)
            dn.store(p)
            out[fused] = p.cpu().numpy()
        else:
            proc.cpsdDenoise(iterations=2, d=d, fused=False)
            out[fused] = proc.graph.pos.cpu().numpy()
    dev = np.linalg.norm(out[True] - out[False], axis=1) / bbox
    report(f"rscale {rscale}: exact {np.mean(dev == 0):.4f} p99.9 {np.percentile(dev, 99.9):.3g} max {dev.max():.3g}")
    assert np.percentile(dev, 99.9) <= 1e-6 and np.median(dev) <= 1e-7, (np.percentile(dev, 99.9), np.median(dev))


@pytest.mark.parametrize("rscale", [1.0, 1.8], ids=["r_d_lds_slots", "r_1.8d_global_slots"])
def test_cpsd_fused_equals_op_by_op_large_cloud(gpu, rscale):
    """The fused driver on a cloud past 2^18 rows (300k bunny-sampled points, bench.make_cloud): there the member
    slots grow into global memory once a selection needs more than 16 (r = 1.8 d: ~50 members), at r = d they stay in
    LDS.  One iteration against the op-by-op drop-in path within 1e-6 x bbox."""
    from bench import make_cloud
    pos0, n0, _ = make_cloud(300_000, 7, gpu)
    bbox = float(torch.linalg.norm(pos0.max(0).values - pos0.min(0).values))
    d = 2 * float(Processor(Pointcloud(pos0.clone(), n0.clone()), k_hint=16).meanEdgeLength())
    out = {}
    for fused in (True, False):
        proc = Processor(Pointcloud(pos0.clone(), n0.clone()), k_hint=16)
        if rscale != 1.0:
            proc.getMartinFeatureDecomposition = (lambda f: (lambda r, rho=0.9: f(r * rscale, rho)))(
                proc.getMartinFeatureDecomposition)
        if fused:
            import pcd_native as nat
            dn = proc._fused_for(8)
            dn.load(proc.graph.pos, proc.graph.n)
            dn.cpsd_iterate(nat.make_cpsd_params(r=d * rscale, d=d), 1)
            p = torch.empty_like(proc.graph.pos)
            dn.store(p)
            out[fused] = p.cpu().numpy()
        else:
            proc.cpsdDenoise(iterations=1, d=d, fused=False)
            out[fused] = proc.graph.pos.cpu().numpy()
    dev = np.linalg.norm(out[True] - out[False], axis=1) / bbox
    report(f"large rscale {rscale}: exact {np.mean(dev == 0):.4f} p99.9 {np.percentile(dev, 99.9):.3g} max {dev.max():.3g}")
    assert np.percentile(dev, 99.9) <= 1e-6 and np.median(dev) <= 1e-7, (np.percentile(dev, 99.9), np.median(dev))
