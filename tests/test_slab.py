"""Spatial-slab multi-rank path on the CPU: the partition, and the driver with world_size 1 and 2
(gloo) over the oracle engine (tests/slab_cpu_engine.py), checked against the single-process oracle loop."""
import os
import socket

import numpy as np
import pytest
import torch

import pcd_native as nat
from oracle import pcd_oracle as O
from pcd_slab import LocalTransport, SlabDenoiser, SlabPlan, TorchTransport, gather_global
from slab_cpu_engine import CpuSlabEngine

K, KU, ITERS = 16, 8, 2


def _cloud(n=2500, seed=5):
    from bench import make_cloud
    pos, nrm, _ = make_cloud(n, seed, torch.device("cpu"))
    return pos, nrm


def _halo(pos, k, factor=3.0):
    _, d = O.FrozenKNN(pos.numpy()).query(pos.numpy(), k)
    return factor * float(np.max(d[:, -1]))


def _params(pos):
    d = 2 * O.mean_edge_length(pos.numpy(), O.FrozenKNN(pos.numpy()))
    return nat.make_params(k=K, k_update=KU, d=d), d


def _reference(pos, nrm, d):
    p, n = pos.numpy().copy(), nrm.numpy().copy()
    knn = O.FrozenKNN(p)
    for _ in range(ITERS):
        p, n, _ = O.denoise_iteration(p, n, knn, d, K, KU)
    return p, n


def test_plan_partition_and_halo():
    pos, _ = _cloud()
    world = 3
    halo = _halo(pos, K)
    plan = SlabPlan.build(pos, world, halo)
    counts = torch.bincount(plan.owner, minlength=world)
    assert counts.max() - counts.min() <= 1
    assert plan.lo == sorted(plan.lo) and all(a <= b for a, b in zip(plan.lo, plan.hi))
    nbr, _ = O.FrozenKNN(pos.numpy()).query(pos.numpy(), K)
    for r in range(world):
        loc = set(plan.local[r].tolist())
        own = torch.nonzero(plan.owner == r).flatten()
        assert set(own.tolist()) <= loc
        # every owned point's exact k-neighbourhood of the snapshot is local
        assert set(np.unique(nbr[own.numpy()]).tolist()) <= loc
        for src in range(world):
            if src == r:
                continue
            t = plan.transfer(src, r)
            assert (plan.owner[t] == src).all() and set(t.tolist()) <= loc
            assert torch.equal(t, torch.sort(t).values)
    lo, hi = plan.coverage(0)
    assert lo[plan.axis] < -1e37 and hi[plan.axis] == pytest.approx(plan.hi[0] + halo)


def test_slab_world1_matches_oracle():
    pos, nrm = _cloud(1500)
    params, d = _params(pos)
    sd = SlabDenoiser(pos, nrm, max(K, KU), transport=LocalTransport(), halo=_halo(pos, K),
                      engine_factory=CpuSlabEngine)
    sd.iterate(params, ITERS)
    sd.check()
    p, n = gather_global(sd.owned_state(), pos.size(0), sd.t)
    rp, rn = _reference(pos, nrm, d)
    np.testing.assert_array_equal(p.numpy(), rp)
    np.testing.assert_array_equal(n.numpy(), rn)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, halo_scale, opts=None):
    from slab_cpu_engine import CpuSlabEngineDiag
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    opts = dict(opts or {})
    rebalance_after = opts.pop("rebalance_after", None)
    engine = CpuSlabEngineDiag if opts.pop("diagnostics", False) else CpuSlabEngine
    try:
        pos, nrm = _cloud()
        params, _ = _params(pos)
        tr = TorchTransport()
        # only the coordinator (rank 0) hands in the cloud; the others receive their slab + halo from it
        sd = SlabDenoiser(pos if rank == 0 else None, nrm if rank == 0 else None, max(K, KU), transport=tr, halo=_halo(pos, K) * halo_scale,
                          engine_factory=engine, **opts)
        owned0 = sd.owned_global.numel()
        halo0 = sd.halo
        if rebalance_after is None:
            sd.iterate(params, ITERS)
        else:
            sd.iterate(params, rebalance_after)
            sd.rebalance(class_weights=(1.0, 3.0, 5.0))
            sd.iterate(params, ITERS - rebalance_after)
        err = 0
        try:
            sd.check()
        except nat.PcdError:
            err = 1
        flag = torch.tensor([err], dtype=torch.int64)
        dist.all_reduce(flag)
        p, n = gather_global(sd.owned_state(), pos.size(0), tr)
        owned = torch.tensor([owned0, sd.owned_global.numel()], dtype=torch.int64)
        allo = [torch.zeros_like(owned) for _ in range(world)]
        dist.all_gather(allo, owned)
        if rank == 0:
            np.savez(out_path, pos=p.numpy(), n=n.numpy(), err=int(flag), halo=sd.halo_points, replans=sd.replans,
                     final_halo=sd.halo, halo0=halo0, owned=torch.stack(allo).numpy(),
                     log=np.array([repr(x) for x in sd.replan_log]))
    finally:
        dist.destroy_process_group()


def _run_world(tmp_path, halo_scale, world=2, opts=None):
    import torch.multiprocessing as mp
    out = str(tmp_path / f"slab_{world}_{halo_scale}.npz")
    mp.spawn(_worker, args=(world, _free_port(), out, halo_scale, opts), nprocs=world, join=True)
    return np.load(out)


def _run_world2(tmp_path, halo_scale, opts=None):
    return _run_world(tmp_path, halo_scale, 2, opts)


def _assert_matches_oracle(res):
    pos, nrm = _cloud()
    _, d = _params(pos)
    rp, rn = _reference(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    # identical per-point arithmetic; only the f64 order of the global flat-centre sum differs across ranks
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


def test_slab_world2_gloo_matches_oracle(tmp_path):
    res = _run_world2(tmp_path, 1.0)
    assert int(res["err"]) == 0 and int(res["halo"]) > 0
    pos, nrm = _cloud()
    _, d = _params(pos)
    rp, rn = _reference(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    # identical per-point arithmetic; only the f64 order of the global flat-centre sum differs across ranks
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


def test_slab_world2_thin_halo_is_reported(tmp_path):
    """With the coverage checks off (check_every=0) a thin halo is reported by check(), never silently used."""
    res = _run_world2(tmp_path, 1e-4, {"check_every": 0})
    assert int(res["err"]) == 2          # both ranks hold a slab face the k-balls cross


def test_slab_world2_thin_halo_replans_and_matches_oracle(tmp_path):
    """A deliberately thin halo (1/20 of the estimate): the driver detects the k-balls leaving the slab, restores the
    checkpoint, widens the halo (x 3 per re-plan), re-plans both ranks from the frozen snapshot and replays -- and
    the result is the single-process oracle's."""
    res = _run_world2(tmp_path, 0.05, {"check_every": 1, "halo_growth": 3.0})
    assert int(res["err"]) == 0
    assert int(res["replans"]) >= 1
    assert float(res["final_halo"]) == pytest.approx(float(res["halo0"]) * 3.0 ** int(res["replans"]), rel=1e-6)
    _assert_matches_oracle(res)


def test_slab_world2_thin_halo_grows_by_the_measured_reach(tmp_path):
    """With the coverage diagnostics (the engine reports how far the farthest k-ball reached past the band box, as
    libpcd's pcd_denoiser_coverage_excess does) a re-plan grows the band by 1.5 x that reach (at least x 1.1) instead
    of x halo_growth: one re-plan covers it, the final band is far below the x 3 growth, and the result is the
    oracle's."""
    import ast
    res = _run_world2(tmp_path, 0.05, {"check_every": 1, "halo_growth": 3.0, "diagnostics": True})
    assert int(res["err"]) == 0
    assert int(res["replans"]) == 1, list(res["log"])       # (x 3 growth from the same start: 2 re-plans)
    log = ast.literal_eval(str(res["log"][0]))
    assert log["band_failed"] and not log["sphere_failed"] and log["band_excess"] > 0
    halo0 = float(res["halo0"])
    assert float(res["final_halo"]) == pytest.approx(max(1.1 * halo0, halo0 + 1.5 * log["band_excess"]), rel=1e-6)
    _assert_matches_oracle(res)


def test_slab_world2_rebalance_by_cost_matches_oracle(tmp_path):
    """rebalance() after the first iteration re-cuts the slabs by class cost (edge 3x, corner 5x a flat point):
    ownership moves between ranks and the run still equals the oracle's."""
    res = _run_world2(tmp_path, 1.0, {"rebalance_after": 1})
    assert int(res["err"]) == 0
    owned = res["owned"]                  # per rank: (before, after)
    assert (owned[:, 0] != owned[:, 1]).any() and owned[:, 1].sum() == owned[:, 0].sum()
    _assert_matches_oracle(res)


def test_slab_world2_rebalance_verifies_pending_iterations(tmp_path):
    """rebalance() in the middle of a check window (check_every=2, one unchecked iteration) on a thin halo: the
    pending iterations are verified first -- the coverage miss re-plans and replays them -- so the state carried into
    the cost-weighted cut is exact and the run still equals the oracle's."""
    res = _run_world2(tmp_path, 0.05, {"check_every": 2, "halo_growth": 3.0, "rebalance_after": 1})
    assert int(res["err"]) == 0
    assert int(res["replans"]) >= 1
    _assert_matches_oracle(res)


def test_plan_weighted_cut():
    pos, _ = _cloud()
    w = torch.ones(pos.size(0), dtype=torch.float32)
    key = pos[:, int(torch.argmax(pos.max(0).values - pos.min(0).values))]
    w[key > key.median()] = 3.0           # the upper half costs 3x: rank 1 of 2 gets fewer points
    plan = SlabPlan.build(pos, 2, 0.01, weights=w)
    counts = torch.bincount(plan.owner, minlength=2)
    assert counts[1] < counts[0]
    load = torch.zeros(2).index_add_(0, plan.owner, w)
    assert abs(float(load[0] - load[1])) <= 2 * 3.0 + 1e-4     # the cut straddles at most one point: 2 w_max


def test_slab_world4_gloo_matches_oracle(tmp_path):
    """Four ranks: the two interior slabs exchange halos with a neighbour on either side (the 8-GPU layout's
    interior case), and both all-reduces span every rank."""
    res = _run_world(tmp_path, 1.0, 4)
    assert int(res["err"]) == 0 and int(res["halo"]) > 0
    pos, nrm = _cloud()
    _, d = _params(pos)
    rp, rn = _reference(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


def test_bench_refuses_more_gpus_than_the_box_has():
    """`bench.py --gpus N` with fewer than N GPUs (none here) stops before any rank starts, unless told to rehearse
    on one GPU."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has the GPUs")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1"], cwd=root,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr


def _bunny_mesh():
    m = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                             "stanford_bunny_mesh.npz"))
    v, f = m["v"].astype(np.float64), m["f"].astype(np.int64)
    cr = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 1]])
    fn = cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)
    # a perturbed field of target normals, so the sweeps move the vertices
    rng = np.random.default_rng(4)
    fn = fn + 0.2 * rng.standard_normal(fn.shape)
    return v, f, fn / np.linalg.norm(fn, axis=1, keepdims=True)


def _mesh_worker(rank, world, port, out_path, sweeps):
    import torch.distributed as dist
    from pcd_slab import MeshSlabs
    from slab_cpu_engine import CpuMeshEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v, f, fn = _bunny_mesh() if rank == 0 else (None, None, None)
        ms = MeshSlabs(v, f, fn, transport=TorchTransport(), engine_factory=CpuMeshEngine)
        ms.update(sweeps)
        ids, pv = ms.owned_state()
        np.savez(f"{out_path}_{rank}.npz", ids=ids.numpy(), v=pv.numpy(), halo=ms.halo_rows)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_mesh_slabs_match_one_process_bitwise(tmp_path, world):
    """Mesh.updateVertices over vertex slabs (pcd_slab.MeshSlabs): gloo ranks, the oracle's sweep as the
    engine, every owned vertex equal to the single-process oracle bit for bit after 3 sweeps -- each owned vertex
    sums all of its faces in the reference's order and reads the previous sweep's halo rows."""
    import torch.multiprocessing as mp
    sweeps = 3
    prefix = str(tmp_path / f"mesh{world}")
    mp.spawn(_mesh_worker, args=(world, _free_port(), prefix, sweeps), nprocs=world, join=True)
    v, f, fn = _bunny_mesh()
    ref = O.mesh_update(v, f, fn, k=sweeps)
    got = np.full_like(ref, np.nan)
    halos = []
    for r in range(world):
        z = np.load(f"{prefix}_{r}.npz")
        got[z["ids"]] = z["v"]
        halos.append(int(z["halo"]))
    assert min(halos) > 0
    np.testing.assert_array_equal(got, ref)
