"""GPU parity at the BASELINE configurations' sizes (BASELINE.json configs[0], [2], [3]).

* configs[3] headline workload (10M bunny-sampled points, sigma = 0.005 x bbox, k = 32, k_u = 8): 25 iterations of the
  shipped fused loop (anchored kNN + LDS row windows) against the reference path of the same library (every kNN an
  unseeded grid search, every neighbour row read from global memory), compared bit for bit after EVERY iteration --
  positions, normals and classes.  Any kNN list that differed would change the state (the loop is chaotic), so this
  pins the anchored lists, the re-anchoring searches and the window reads at the size the bench times.
* a 200k-point sample of the same workload: one iteration against the CPU oracle (classes >= 99.8 %, p99 position
  deviation <= 1e-5 x bbox, median <= 1e-7 x bbox -- the tolerances of test_gpu_parity's single-iteration check).
* configs[0] (bunny vertices, sigma = 0.003 x bbox, seed 0, k = 16, 5 iterations): per-iteration Chamfer distance to the
  clean bunny against the oracle's, within 3x the oracle's own sensitivity to a 1e-6 perturbation of its input normals
  (measured in the test) plus 0.2 %.
* configs[2] (170k-point substitute for the missing armadillo blob, k = 32, 20 iterations): first iteration against
  the oracle, 20 iterations bitwise anchored-vs-reference, and the Chamfer trajectory's first three values against the
  oracle.
"""
import numpy as np
import pytest
import torch

import pcd_native as nat
from oracle import pcd_oracle as O
from Pointcloud.Modules.Object import Pointcloud, sample_surface
from Pointcloud.Modules.Processor import Processor
from conftest import report

pytestmark = pytest.mark.gpu


def bunny():
    import os
    m = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                             "stanford_bunny_mesh.npz"))
    return m["v"].astype(np.float32), m["f"].astype(np.int64)


def bunny_cloud(n, seed, sigma_frac):
    """The bench's workload (bench.make_cloud) sampled on the CPU so it is reproducible everywhere."""
    v, f = bunny()
    g = torch.Generator().manual_seed(seed)
    pos, nrm = sample_surface(torch.from_numpy(v), torch.from_numpy(f), n, generator=g)
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    pos = pos + sigma_frac * diag * torch.randn(pos.shape, generator=g)
    return pos.contiguous(), nrm.contiguous()


def run_pair(pos, nrm, k, iterations, dev, check_every=True):
    """Shipped loop vs the library's reference path on one cloud; returns the redo rows per iteration.  Both end
    with pcd_denoiser_check (inside store): a bad list entry would raise."""
    pc = Pointcloud(pos.to(dev), nrm.to(dev))
    proc = Processor(pc, k_hint=k)
    d = 2 * float(proc.meanEdgeLength())
    params = nat.make_params(k=k, k_update=8, d=d)
    a = proc._fused_for(k)
    b = nat.FusedDenoiser(a.grid, k)   # the same snapshot index: exact distance ties break by its rank order
    a.load(proc.graph.pos, proc.graph.n)
    b.load(proc.graph.pos, proc.graph.n)
    b.set_seeding(False)
    b.set_windows(False)
    N = pos.shape[0]
    bufs = [(torch.empty((N, 3), device=dev), torch.empty((N, 3), device=dev),
             torch.empty(N, dtype=torch.int64, device=dev)) for _ in range(2)]
    redo = []
    for it in range(1, iterations + 1):
        a.iterate(params, 1)
        b.iterate(params, 1)
        redo.append(a.redo_rows())
        if check_every or it == iterations:
            for fused, (p, n, c) in zip((a, b), bufs):
                fused.store(p, n, c)
            (pa, na, ca), (pb, nb, cb) = bufs
            bad = (pa != pb).any(1) | (na != nb).any(1) | (ca != cb)
            assert not bool(bad.any()), (f"iteration {it}: {int(bad.sum())} of {N} rows differ between the anchored "
                                         f"loop and the unseeded reference path")
    a.check()
    b.check()
    return redo, d


def test_headline_10m_25_iterations_bitwise(gpu):
    """BASELINE configs[3] at full size: 25 iterations, state compared bitwise after every one."""
    pos, nrm = bunny_cloud(10_000_000, 2, 0.005)
    redo, _ = run_pair(pos, nrm, 32, 25, gpu)
    # the re-anchoring path is exercised on every iteration (the dense first one re-anchors every row)
    assert redo[0] == 10_000_000 and min(redo[1:]) > 10_000, redo


def test_headline_workload_2m_40_iterations_bitwise(gpu):
    """Past the re-anchoring peak (iterations 25-40 re-anchor ~9 % of the rows a step): 2M points of the
    headline workload for 40 anchored iterations, state bitwise against the reset-seed path after every one."""
    pos, nrm = bunny_cloud(2_000_000, 2, 0.005)
    redo, _ = run_pair(pos, nrm, 32, 40, gpu)
    assert redo[0] == 2_000_000 and min(redo[1:]) > 0, redo
    assert max(redo[20:]) > 0.02 * 2_000_000, redo        # the peak window really re-anchors at scale


def test_config5_80m_one_gpu_bitwise(gpu):
    """BASELINE configs[4]'s whole 80M-point cloud (the bench's slab workload: bench.make_cloud seed 3, sampled on
    the device) on ONE MI355X: 3 anchored iterations against the reset-seed path (every kNN an unseeded grid
    search, no LDS windows), state bitwise after every iteration, and the device error word checked at the end
    (store() runs pcd_denoiser_check: no invalid list entry).  ~75 GB of device state for the pair."""
    from bench import make_cloud
    pos, nrm, _ = make_cloud(80_000_000, 3, gpu)
    redo, _ = run_pair(pos, nrm, 32, 3, gpu)
    assert redo[0] == 80_000_000 and min(redo[1:]) > 0, redo


def _one_iteration_vs_oracle(pos, nrm, k, dev):
    p0, n0 = pos.numpy(), nrm.numpy()
    knn = O.FrozenKNN(p0)
    d = 2 * O.mean_edge_length(p0, knn)
    rpos, rn, rcls = O.denoise_iteration(p0, n0, knn, d, k, 8)
    pc = Pointcloud(pos.to(dev), nrm.to(dev))
    proc = Processor(pc, k_hint=k)
    fused = proc._fused_for(k)
    fused.load(proc.graph.pos, proc.graph.n)
    fused.iterate(nat.make_params(k=k, k_update=8, d=d), 1)
    N = len(p0)
    gp = torch.empty((N, 3), device=dev); gn = torch.empty((N, 3), device=dev)
    gc = torch.empty(N, dtype=torch.int64, device=dev)
    fused.store(gp, gn, gc)
    agree = float((gc.cpu().numpy() == rcls).mean())
    bbox = float(np.linalg.norm(p0.max(0) - p0.min(0)))
    dev_pos = np.linalg.norm(gp.cpu().numpy() - rpos, axis=1) / bbox
    report(f"{N} points, 1 iteration vs the oracle: classes {agree:.6f} median {np.median(dev_pos):.3g} "
          f"p99 {np.percentile(dev_pos, 99):.3g} p99.9 {np.percentile(dev_pos, 99.9):.3g} max {dev_pos.max():.3g}")
    # the oracle restates NVT1 to the bit (MKL-exact eigh, torch's norm), so only kNN near-ties between the fp32 grid
    # and the f64 KD-tree, NVT2's Jacobi at an argmax margin and the flat step's exp / centre rounding remain
    # (measured at 170k / 200k / 1M: classes >= 0.999999, median 0, p99 <= 5.1e-8, p99.9 <= 2.0e-7)
    assert agree >= 0.99999, agree
    assert np.median(dev_pos) == 0 and np.percentile(dev_pos, 99) <= 1e-6 and np.percentile(dev_pos, 99.9) <= 1e-5, \
        (np.median(dev_pos), np.percentile(dev_pos, 99), np.percentile(dev_pos, 99.9))


def test_headline_workload_sample_one_iteration_vs_oracle(gpu):
    """A 200k-point sample of the configs[3] workload: one fused iteration against the CPU oracle."""
    pos, nrm = bunny_cloud(200_000, 2, 0.005)
    _one_iteration_vs_oracle(pos, nrm, 32, gpu)


def test_headline_workload_1m_one_iteration_vs_oracle(gpu):
    """The bench's `parity` sample (bench.cpu_baseline: 1M points of the headline workload, make_cloud seed 99 drawn
    on the host): one fused iteration against the CPU oracle at the one-iteration gate."""
    from bench import make_cloud
    pos, nrm, _ = make_cloud(1_000_000, 99, torch.device("cpu"))
    _one_iteration_vs_oracle(pos, nrm, 32, gpu)


def bunny_config1():
    """configs[0]: the bunny's vertices + isotropic noise sigma = 0.003 x bbox (torch seed 0); normals = area-weighted
    vertex normals of the clean mesh ((0, 0, 1) for the mesh's unreferenced vertices)."""
    v, f = bunny()
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    cr = np.cross(b - a, c - a)
    vn = np.zeros_like(v)
    for kk in range(3):
        np.add.at(vn, f[:, kk], cr)
    nn = np.linalg.norm(vn, axis=1, keepdims=True)
    vn = np.where(nn > 0, vn / np.maximum(nn, 1e-30), np.array([[0, 0, 1.0]])).astype(np.float32)
    diag = float(np.linalg.norm(v.max(0) - v.min(0)))
    g = torch.Generator().manual_seed(0)
    pos = (torch.from_numpy(v) + 0.003 * diag * torch.randn(v.shape, generator=g)).numpy().astype(np.float32)
    return v, pos, vn


def test_config1_bunny_k16_five_iterations(gpu):
    gt, pos, n0 = bunny_config1()
    cds = {}
    for tag, nin in (("ref", n0), ("pert", n0 + 1e-6 * np.random.default_rng(1).standard_normal(n0.shape)
                                   .astype(np.float32))):
        knn = O.FrozenKNN(pos)
        d = 2 * O.mean_edge_length(pos, knn)
        p, n = pos.copy(), nin.copy()
        cds[tag] = []
        for _ in range(5):
            p, n, _ = O.denoise_iteration(p, n, knn, d, 16, 8)
            cds[tag].append(float(O.chamfer(gt, p).mean()))
    pc = Pointcloud(torch.from_numpy(pos.copy()).to(gpu), torch.from_numpy(n0.copy()).to(gpu))
    proc = Processor(pc, k_hint=16)
    dd = 2 * float(proc.meanEdgeLength())
    assert abs(dd - d) <= 1e-5 * d
    got = []
    for _ in range(5):
        proc.denoise(iterations=1, k=16, k_update=8, d=d)
        got.append(float(O.chamfer(gt, pc.v.cpu().numpy()).mean()))
    ref, pert = np.array(cds["ref"]), np.array(cds["pert"])
    env = 3 * np.abs(ref - pert) + 2e-3 * ref
    assert np.all(np.abs(np.array(got) - ref) <= env), (got, list(ref), list(env))
    assert got[-1] < float(O.chamfer(gt, pos).mean())       # denoising lowered the error


def test_config3_170k_k32_twenty_iterations(gpu):
    """configs[2] substitute (armadillo_gaus_n3.obj is a missing blob): 170k bunny samples + sigma = 0.003 x bbox."""
    pos, nrm = bunny_cloud(170_000, 1, 0.003)
    _one_iteration_vs_oracle(pos, nrm, 32, gpu)
    redo, d = run_pair(pos, nrm, 32, 20, gpu, check_every=True)
    assert redo[0] == 170_000
    # Chamfer trajectory vs the oracle for the first 3 iterations (before the chaos of SURVEY §0 sets in)
    v, _ = bunny()
    p0, n0 = pos.numpy(), nrm.numpy()
    knn = O.FrozenKNN(p0)
    p, n = p0.copy(), n0.copy()
    pc = Pointcloud(pos.to(gpu), nrm.to(gpu))
    proc = Processor(pc, k_hint=32)
    for _ in range(3):
        p, n, _ = O.denoise_iteration(p, n, knn, d, 32, 8)
        proc.denoise(iterations=1, k=32, k_update=8, d=d)
        c_ref = float(O.chamfer(v, p).mean())
        c_gpu = float(O.chamfer(v, pc.v.cpu().numpy()).mean())
        assert abs(c_gpu - c_ref) <= 2e-3 * c_ref, (c_gpu, c_ref)


def test_k1_only_timing_level(gpu):
    """pcd_denoiser_set_timing(2), the bench's timed region: one slot (K1's ms), consistent with the full split's K1
    slots on a replay of the same iterations, and timing changes no result (state bitwise equal either way)."""
    pos, nrm = bunny_cloud(400_000, 5, 0.005)
    pc = Pointcloud(pos.to(gpu), nrm.to(gpu))
    proc = Processor(pc, k_hint=32)
    params = nat.make_params(k=32, k_update=8, d=2 * float(proc.meanEdgeLength()))
    fused = proc._fused_for(32)
    out = []
    for level in (2, True):
        fused.load(proc.graph.pos, proc.graph.n)
        fused.reset_seed()
        fused.iterate(params, 3)
        fused.set_timing(level)
        fused.iterate(params, 5)
        slots = fused.timing()
        fused.set_timing(False)
        p, n = torch.empty_like(pc.v), torch.empty_like(pc.v)
        fused.store(p, n)
        out.append((slots, p, n))
    (k1, p2, n2), (full, p1, n1) = out
    assert len(k1) == 1 and k1[0] > 0, k1
    assert len(full) >= len(nat.FusedDenoiser.TIMING_SLOTS), full   # (+ the trailing "-" slot)
    k1_full = sum(full[:4])
    report(f"K1 ms: K1-only events {k1[0]:.4f}, full split {k1_full:.4f} (400k points, iterations 4-8)")
    assert 0.5 * k1_full < k1[0] < 2.0 * k1_full
    assert torch.equal(p1, p2) and torch.equal(n1, n2)
