"""Spatial slabs on the GPU: the staged HIP engine against the one-GPU fused loop, with one rank,
with two ranks sharing the box's GPU over libpcd's host-callback transport on a gloo group, and -- where at least two
GPUs are visible -- two ranks on two GPUs over libpcd's own RCCL communicator (skipped on a one-GPU box, the driver's
8-GPU bench exercises it at scale).  Only rank 0 (the coordinator) ever holds the whole cloud."""
import os
import socket

import numpy as np
import pytest
import torch

import pcd_native as nat
from pcd_slab import LocalTransport, SlabDenoiser, TorchTransport, gather_global, default_halo
from conftest import report

K, KU, ITERS = 32, 8, 3


def _cloud(dev, n=60000, seed=11):
    from bench import make_cloud
    pos, nrm, _ = make_cloud(n, seed, dev)
    return pos, nrm


def _d(pos):
    from Pointcloud.Modules.Object import Pointcloud
    from Pointcloud.Modules.Processor import Processor
    return 2 * float(Processor(Pointcloud(pos.clone())).meanEdgeLength())


def _params(d, jacobi=False):
    if not jacobi:
        return nat.make_params(k=K, k_update=KU, d=d)
    # the thesis driver's composition (PostProcessing.ipynb:1069-1090): Jacobi across classes + global clamp
    ph = ((0, nat.STEP_FLAT, 1.0), (1, nat.STEP_FEATURE, 0.2), (2, nat.STEP_FEATURE, 1.0))
    return nat.make_params(k=K, k_update=KU, d=d * 20000, phases=ph, jacobi=True, clamp_global=d)


def _fused(pos, nrm, d, jacobi=False, iters=ITERS):
    g = nat.Grid(pos, k_hint=K)
    fd = nat.FusedDenoiser(g, max(K, KU))
    fd.load(pos, nrm)
    fd.iterate(_params(d, jacobi), iters)
    p, n = torch.empty_like(pos), torch.empty_like(nrm)
    fd.store(p, n)
    return p.cpu().numpy(), n.cpu().numpy()


@pytest.mark.gpu
def test_hip_slab_world1_is_the_fused_loop(gpu):
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    sd = SlabDenoiser(pos, nrm, max(K, KU), transport=LocalTransport(), k_hint=K)
    sd.iterate(nat.make_params(k=K, k_update=KU, d=d), ITERS)
    sd.check()
    p, n = gather_global(sd.owned_state(), pos.size(0), sd.t)
    rp, rn = _fused(pos, nrm, d)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)
    np.testing.assert_array_equal(n.cpu().numpy(), rn)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, cloud_path, d, backend="gloo", jacobi=False, native=None, sq=0.999,
            readset=True):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # the control group is always gloo; backend "rccl" = libpcd's own RCCL communicator as the data plane (one GPU
    # per rank), "gloo" = its host-callback transport (ranks sharing the box's GPU)
    dev = torch.device("cuda", rank if backend == "rccl" else 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos = nrm = None
        if rank == 0:                   # only the coordinator holds the cloud
            c = np.load(cloud_path)
            pos, nrm = torch.from_numpy(c["pos"]).to(dev), torch.from_numpy(c["n"]).to(dev)
        tr = TorchTransport(rccl=backend == "rccl")
        # the default halo priced for the drift of the whole run (step bound d, ITERS iterations: cut_spheres)
        sd = SlabDenoiser(pos, nrm, max(K, KU), transport=tr, k_hint=K, native=native, sphere_quantile=sq,
                          step_bound=d, horizon=ITERS)
        if native is not False:
            assert sd.comm.info() == {"world": world, "rank": rank,
                                      "transport": "rccl" if backend == "rccl" else "host"}
        if sd.native and not readset:
            sd.e.fused.set_readset(False)
        sd.iterate(_params(d, jacobi), ITERS)
        sd.check()
        rs = sd.e.readset_stats() if sd.native else (0, 0, 0)
        p, n = gather_global(sd.owned_state(), sd.n_total, tr)
        if rank == 0:
            np.savez(out_path, pos=p.numpy(), n=n.numpy(), halo=sd.halo_points, replans=sd.replans,
                     spheres=0 if sd.plan.spheres is None else int(sd.plan.spheres.ids.numel()),
                     rs_iters=rs[0], rs_recv=rs[2])
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_hip_slab_world2_matches_one_gpu(gpu, tmp_path):
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    out, cloud = str(tmp_path / "slab2.npz"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker, args=(2, _free_port(), out, cloud, d), nprocs=2, join=True)
    res = np.load(out)
    assert int(res["halo"]) > 0
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    # same kernels and tie-breaks; only the f64 summation order of the global flat centre differs
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_hip_slab_world1_staged_is_the_fused_loop(gpu):
    """The Python-driven stage sequence (native=False: pcd_denoiser_stage + pack/unpack), the reference the one-call
    path is checked against, is itself the fused loop bit for bit."""
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    sd = SlabDenoiser(pos, nrm, max(K, KU), transport=LocalTransport(), k_hint=K, native=False)
    sd.iterate(nat.make_params(k=K, k_update=KU, d=d), ITERS)
    sd.check()
    p, n = gather_global(sd.owned_state(), pos.size(0), sd.t)
    rp, rn = _fused(pos, nrm, d)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)
    np.testing.assert_array_equal(n.cpu().numpy(), rn)


@pytest.mark.gpu
@pytest.mark.parametrize("jacobi", [False, True], ids=["gauss_seidel", "jacobi"])
def test_hip_slab_world2_one_call_equals_staged(gpu, tmp_path, jacobi):
    """pcd_slab_iterate (one library call per iteration: its exchanges on a stream of their own, overlapped with the
    rows whose k-ball stays inside the owned slab; here over the host-callback transport on gloo) against the same
    stages driven one by one from Python: bit-identical."""
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    cloud = str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    got = {}
    for native in (True, False):
        out = str(tmp_path / f"slab2_{native}.npz")
        mp.spawn(_worker, args=(2, _free_port(), out, cloud, d, "gloo", jacobi, native), nprocs=2, join=True)
        got[native] = np.load(out)
    assert int(got[True]["halo"]) > 0
    np.testing.assert_array_equal(got[True]["pos"], got[False]["pos"])
    np.testing.assert_array_equal(got[True]["n"], got[False]["n"])


@pytest.mark.gpu
def test_hip_slab_world4_readset_equals_every_row(gpu, tmp_path):
    """The read-set exchange (pcd_denoiser_set_readset, the default: after the kNN each rank asks its peers for the
    halo rows its lists hold, and every exchange of the iteration moves only those) against every halo row in every
    exchange: bit-identical, with fewer rows moved than held."""
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    cloud = str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    got = {}
    for rs in (True, False):
        out = str(tmp_path / f"slab4_rs{rs}.npz")
        mp.spawn(_worker, args=(4, _free_port(), out, cloud, d, "gloo", False, None, 0.999, rs), nprocs=4, join=True)
        got[rs] = np.load(out)
    assert int(got[True]["replans"]) == 0 and int(got[False]["replans"]) == 0
    assert int(got[True]["rs_iters"]) == ITERS and int(got[False]["rs_iters"]) == 0
    read = int(got[True]["rs_recv"]) / ITERS
    report(f"read-set exchange, rank 0: {read:.0f} of {int(got[True]['halo'])} held halo rows moved per iteration")
    assert 0 < read < int(got[True]["halo"])
    np.testing.assert_array_equal(got[True]["pos"], got[False]["pos"])
    np.testing.assert_array_equal(got[True]["n"], got[False]["n"])


@pytest.mark.gpu
def test_hip_slab_world4_matches_one_gpu(gpu, tmp_path):
    """Four ranks sharing the GPU over gloo: two interior slabs exchange halos with a neighbour on either side,
    as the interior ranks of the 8-GPU run do."""
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    out, cloud = str(tmp_path / "slab4.npz"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker, args=(4, _free_port(), out, cloud, d), nprocs=4, join=True)
    res = np.load(out)
    assert int(res["halo"]) > 0
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


def _worker_owned(rank, world, port, out_prefix, cloud_path, d, halo=None, iters=ITERS, check_every=1,
                  rebalance_after=None):
    """Like _worker, but every rank saves its own points (ids, pos, n) -- no all-gather of the whole cloud."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos = nrm = None
        if rank == 0:                   # only the coordinator holds the cloud
            c = np.load(cloud_path)
            pos, nrm = torch.from_numpy(c["pos"]).to(dev), torch.from_numpy(c["n"]).to(dev)
        tr = TorchTransport()
        sd = SlabDenoiser(pos, nrm, max(K, KU), transport=tr, k_hint=K, halo=halo, check_every=check_every)
        del pos, nrm
        owned0 = sd.owned_global.numel()
        if rebalance_after is None:
            sd.iterate(_params(d), iters)
        else:
            sd.iterate(_params(d), rebalance_after)
            sd.rebalance()
            sd.iterate(_params(d), iters - rebalance_after)
        sd.verify()                     # the iterations since the last check (the bench's exactness check)
        sd.check()
        ids, p, n = sd.owned_state()
        np.savez(f"{out_prefix}_{rank}.npz", ids=ids.cpu().numpy(), pos=p.cpu().numpy(), n=n.cpu().numpy(),
                 halo=sd.halo_points, replans=sd.replans, owned=[owned0, ids.numel()])
    finally:
        dist.destroy_process_group()


def _assemble(prefix, world, n):
    pos = np.full((n, 3), np.nan, np.float32)
    nrm = np.full((n, 3), np.nan, np.float32)
    halos, replans = [], []
    for r in range(world):
        z = np.load(f"{prefix}_{r}.npz")
        pos[z["ids"]] = z["pos"]
        nrm[z["ids"]] = z["n"]
        halos.append(int(z["halo"]))
        replans.append(int(z["replans"]))
    return pos, nrm, halos, replans


@pytest.mark.gpu
def test_hip_slab_world8_8m_points_matches_one_gpu(gpu, tmp_path):
    """BASELINE configs[4]'s topology: 8 ranks (6 interior slabs with a halo neighbour on either side) over 8M
    points, sharing the box's GPU over gloo, against the one-GPU fused loop within 1e-6 x bbox."""
    import torch.multiprocessing as mp
    n = 8_000_000
    pos, nrm = _cloud(gpu, n=n, seed=3)
    d = _d(pos)
    prefix, cloud = str(tmp_path / "slab8"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker_owned, args=(8, _free_port(), prefix, cloud, d), nprocs=8, join=True)
    p, nn, halos, _ = _assemble(prefix, 8, n)
    assert not np.isnan(p).any() and min(halos) > 0
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    dev = np.abs(p - rp).max()
    assert dev <= 1e-6 * bbox, dev / bbox
    np.testing.assert_allclose(nn, rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_hip_slab_world8_rebalance_12_iterations_matches_one_gpu(gpu, tmp_path):
    """What the bench's slab mode runs: 8 ranks (sharing the box's GPU over gloo) on 8M points, cut re-balanced by
    class cost after the second iteration (rebalance() on the HIP engine), coverage checked every 10 iterations
    (check_every=10: one checkpoint / verify cycle inside the run, the second at the end), 12 one-call iterations --
    against the one-GPU fused loop within 1e-6 x bbox."""
    import torch.multiprocessing as mp
    n, iters = 8_000_000, 12
    pos, nrm = _cloud(gpu, n=n, seed=3)
    d = _d(pos)
    prefix, cloud = str(tmp_path / "reb8"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker_owned, args=(8, _free_port(), prefix, cloud, d, None, iters, 10, 2), nprocs=8, join=True)
    p, nn, halos, replans = _assemble(prefix, 8, n)
    owned = np.stack([np.load(f"{prefix}_{r}.npz")["owned"] for r in range(8)])
    assert not np.isnan(p).any() and min(halos) > 0
    assert (owned[:, 0] != owned[:, 1]).any() and owned[:, 1].sum() == n      # the cut moved; every point owned
    rp, rn = _fused(pos, nrm, d, iters=iters)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    dev = np.abs(p - rp).max()
    assert dev <= 1e-6 * bbox, dev / bbox
    np.testing.assert_allclose(nn, rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_rccl_comm_world1_exchange_and_allreduce(gpu):
    """libpcd's own RCCL communicator (pcd_comm_create from pcd_comm_id) on one GPU: a halo route to itself moves
    rows through ncclSend / ncclRecv (pack -> RCCL -> unpack on the library's exchange stream), and the in-place
    scalar all-reduces run through ncclAllReduce."""
    pos, nrm = _cloud(gpu, 5000)
    g = nat.Grid(pos, k_hint=K)
    fd = nat.FusedDenoiser(g, K)
    fd.load(pos, nrm)
    comm = nat.Comm.rccl(1, 0, lambda t: t)
    rows = torch.arange(pos.size(0), dtype=torch.int32, device=gpu)
    before = fd.pack(nat.FIELD_POS, rows)
    src, dst = rows[:1000], rows[2000:3000]
    fd.set_routes([0], [src], [dst])
    fd.halo_exchange(comm, nat.FIELD_POS)
    after = fd.pack(nat.FIELD_POS, rows)
    torch.testing.assert_close(after[2000:3000], before[:1000], rtol=0, atol=0)
    torch.testing.assert_close(after[:2000], before[:2000], rtol=0, atol=0)
    torch.testing.assert_close(after[3000:], before[3000:], rtol=0, atol=0)
    t64 = torch.tensor([1.5, 2.0, -3.0, 4.0], dtype=torch.float64, device=gpu)
    comm.allreduce_(t64, nat.OP_SUM)
    t32 = torch.tensor([7.25], dtype=torch.float32, device=gpu)
    comm.allreduce_(t32, nat.OP_MAX)
    torch.cuda.synchronize()
    assert t64.tolist() == [1.5, 2.0, -3.0, 4.0] and t32.item() == 7.25


@pytest.mark.gpu
def test_rccl_comm_world1_sendrecv_self(gpu):
    """pcd_comm_sendrecv's RCCL branch (the coordinator hand-out and the re-plan gather ride on it): a route to itself
    through ncclSend / ncclRecv, byte counts that are multiples of 4 but not of 16 (odd row counts of 4-byte
    words), every dtype the hand-out moves, and the one-sided forms (send only / receive only skip the other half)."""
    comm = nat.Comm.rccl(1, 0, lambda t: t)
    assert comm.info() == {"world": 1, "rank": 0, "transport": "rccl"}
    g = torch.Generator(device=gpu).manual_seed(11)
    for n, dt in ((1, torch.float32), (1237, torch.float32), (3 * 4001, torch.int32), (999, torch.float64)):
        src = (torch.rand(n, generator=g, device=gpu) * 1e6).to(dt)
        dst = torch.full_like(src, -7)
        comm.sendrecv(0, src, 0, dst)
        torch.cuda.synchronize()
        assert torch.equal(dst, src), (n, dt)
    # empty transfers are a no-op on both sides
    comm.sendrecv(-1, None, -1, None)
    comm.destroy()


def _sendrecv_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = TorchTransport(rccl=False)
        comm = tr.native_comm()
        assert comm.info() == {"world": world, "rank": rank, "transport": "host"}
        # a ring: every rank sends (rank + 1) * 1237 words to its right neighbour and receives its left neighbour's
        right, left = (rank + 1) % world, (rank - 1) % world
        send = torch.arange((rank + 1) * 1237, dtype=torch.int32, device=dev) * (rank + 3)
        recv = torch.full(((left + 1) * 1237,), -1, dtype=torch.int32, device=dev)
        comm.sendrecv(right, send, left, recv)
        torch.cuda.synchronize()
        expect = torch.arange((left + 1) * 1237, dtype=torch.int32, device=dev) * (left + 3)
        ok = torch.equal(recv, expect)
        # one-sided: rank 0 only sends, rank 1 only receives (the coordinator hand-out's pattern)
        if rank == 0:
            comm.sendrecv(1, torch.full((5,), 2.5, device=dev), -1, None)
        elif rank == 1:
            r = torch.zeros(5, device=dev)
            comm.sendrecv(-1, None, 0, r)
            torch.cuda.synchronize()
            ok = ok and bool((r == 2.5).all())
        np.save(f"{out_path}.{rank}.npy", np.array([ok]))
        tr.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_host_comm_world2_sendrecv_ring(gpu, tmp_path):
    """pcd_comm_sendrecv over the host-callback transport between two processes sharing the GPU: a ring exchange of
    unequal odd-sized int32 buffers, then the one-sided send / receive of the coordinator hand-out."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "sr")
    mp.spawn(_sendrecv_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert all(bool(np.load(f"{out}.{r}.npy")[0]) for r in range(2))


@pytest.mark.gpu
def test_hip_slab_world2_thin_halo_replans_and_matches_one_gpu(gpu, tmp_path):
    """A deliberately thin halo (1/20 of default_halo): the first coverage check fails on both ranks, the driver
    restores its checkpoint, widens the halo and re-plans from the frozen snapshot, replays -- and ends where the
    one-GPU fused loop does."""
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    halo = 0.05 * default_halo(pos, K)
    prefix, cloud = str(tmp_path / "thin2"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker_owned, args=(2, _free_port(), prefix, cloud, d, halo), nprocs=2, join=True)
    p, nn, _, replans = _assemble(prefix, 2, pos.size(0))
    assert min(replans) >= 1
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(p, rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(nn, rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_hip_slab_world1_jacobi_is_the_fused_loop(gpu):
    """The Jacobi-across-classes mode with the global clamp through the staged engine (one position refresh per
    iteration instead of one per phase): bit-identical to the fused loop at world 1."""
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    sd = SlabDenoiser(pos, nrm, max(K, KU), transport=LocalTransport(), k_hint=K)
    sd.iterate(_params(d, True), ITERS)
    p, n = gather_global(sd.owned_state(), pos.size(0), sd.t)
    rp, rn = _fused(pos, nrm, d, True)
    np.testing.assert_array_equal(p.cpu().numpy(), rp)
    np.testing.assert_array_equal(n.cpu().numpy(), rn)


@pytest.mark.gpu
def test_hip_slab_world2_jacobi_matches_one_gpu(gpu, tmp_path):
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    out, cloud = str(tmp_path / "slab2j.npz"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker, args=(2, _free_port(), out, cloud, d, "gloo", True), nprocs=2, join=True)
    res = np.load(out)
    rp, rn = _fused(pos, nrm, d, True)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_hip_slab_world2_rccl_two_gpus(gpu, tmp_path):
    """Two ranks on two GPUs over libpcd's RCCL communicator (the bench's multi-GPU data plane; gloo control group);
    needs >= 2 visible GPUs."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL ranks cannot share one device)")
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    out, cloud = str(tmp_path / "slab2r.npz"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker, args=(2, _free_port(), out, cloud, d, "rccl"), nprocs=2, join=True)
    res = np.load(out)
    assert int(res["halo"]) > 0
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_default_halo_covers_knn(gpu):
    pos, _ = _cloud(gpu, 20000)
    h = default_halo(pos, K)
    _, d2 = nat.Grid(pos, k_hint=K).knn(pos, K, with_d2=True)
    assert h >= 2.9 * float(d2[:, -1].max().sqrt())


@pytest.mark.gpu
def test_bench_gpus2_self_launch_rehearsal():
    """`bench.py --gpus 2` launches its two ranks itself (no torchrun), here both on the box's one GPU over libpcd's
    host transport (--rehearse-one-gpu): the line reports two ranks, spatial slabs, libpcd's own view of the world,
    every point owned once and a halo on both ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--rehearse-one-gpu", "--points", "400000", "--steps", "3",
           "--warmup", "3", "--no-extras", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print({k: line[k] for k in ("value", "ms_per_step", "n_gpus")}, line["slab"], line.get("n1"))
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "spatial slabs x2"
    assert line["slab"]["world"] == 2 and line["slab"]["transport"] == "host"
    assert sum(line["slab"]["owned_rows"]) == 800_000 and min(line["slab"]["halo_rows"]) > 0
    assert line["n1"]["points"] == 400_000 and line["value"] > 0


def _mesh_inputs():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    m = np.load(os.path.join(root, "data", "stanford_bunny_mesh.npz"))
    v, f = m["v"].astype(np.float64), m["f"].astype(np.int64)
    cr = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 1]])
    fn = cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)
    fn = fn + 0.2 * np.random.default_rng(4).standard_normal(fn.shape)
    return v, f, fn / np.linalg.norm(fn, axis=1, keepdims=True)


def _mesh_one_gpu(v, f, fn, k, fp32, dev):
    dt, it = (torch.float32, torch.int32) if fp32 else (torch.float64, torch.int64)
    vd = torch.from_numpy(v).to(dev, dt).contiguous()
    fd = torch.from_numpy(f).to(dev, it).contiguous()
    nd = torch.from_numpy(fn).to(dev, dt).contiguous()
    vf, ni = nat.mesh_vta(fd, vd.size(0), out_dtype=it)
    (nat.mesh_update_f32 if fp32 else nat.mesh_update)(vd, fd, nd, vf, ni, k)
    return vd.cpu().numpy()


def _mesh_worker_gpu(rank, world, port, prefix, k, fp32):
    import torch.distributed as dist
    from pcd_slab import MeshSlabs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v, f, fn = _mesh_inputs() if rank == 0 else (None, None, None)
        ms = MeshSlabs(v, f, fn, transport=TorchTransport(), fp32=fp32)
        ms.update(k)
        ids, pv = ms.owned_state()
        np.savez(f"{prefix}_{rank}.npz", ids=ids.cpu().numpy(), v=pv.cpu().numpy(), halo=ms.halo_rows)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("fp32", [False, True], ids=["fp64", "fp32"])
def test_mesh_slabs_world2_equal_one_gpu(gpu, tmp_path, fp32):
    """Mesh.updateVertices over two vertex slabs (pcd_slab.MeshSlabs: the HIP sweep on each rank's local mesh, the
    one-ring halo refreshed through libpcd's communicator -- here its host transport, both ranks on the box's GPU)
    against the one-GPU kernel: every vertex bit-identical after 5 sweeps, in fp64 and in fp32."""
    import torch.multiprocessing as mp
    k = 5
    prefix = str(tmp_path / ("m32" if fp32 else "m64"))
    mp.spawn(_mesh_worker_gpu, args=(2, _free_port(), prefix, k, fp32), nprocs=2, join=True)
    v, f, fn = _mesh_inputs()
    ref = _mesh_one_gpu(v, f, fn, k, fp32, gpu)
    got = np.full_like(ref, np.nan)
    for r in range(2):
        z = np.load(f"{prefix}_{r}.npz")
        assert int(z["halo"]) > 0
        got[z["ids"]] = z["v"]
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
def test_cut_halo_covers_the_snapshot_balls_and_is_thinner(gpu):
    """cut_halo (the default since round 5): every snapshot point's k-ball stays inside its slab widened by the halo,
    and the halo is far thinner than default_halo's sample-maximum estimate (noise outliers price that one)."""
    from pcd_slab import SlabPlan, cut_halo
    pos, _ = _cloud(gpu, 400_000, seed=3)
    world = 4
    h = cut_halo(pos, world, K, margin=1.0)
    hd = default_halo(pos, K)
    plan = SlabPlan.build(pos, world, h)
    _, d2 = nat.Grid(pos, k_hint=K).knn(pos, K, with_d2=True)
    dk = d2[:, -1].sqrt()
    key = pos[:, plan.axis]
    lo = torch.tensor(plan.lo, device=gpu)[plan.owner]
    hi = torch.tensor(plan.hi, device=gpu)[plan.owner]
    top = plan.owner < world - 1
    bot = plan.owner > 0
    assert bool(((key + dk <= hi + h * (1 + 1e-6)) | ~top).all()) and bool(((key - dk >= lo - h * (1 + 1e-6)) | ~bot).all())
    report(f"cut_halo {h:.4g} vs default_halo {hd:.4g} (x{hd / h:.1f})")
    assert h < 0.6 * hd


@pytest.mark.gpu
def test_hip_slab_world4_coverage_spheres_match_one_gpu(gpu, tmp_path):
    """The band halo at the MEDIAN near-face reach (sphere_quantile=0.5): half the points near a cut keep their own
    coverage sphere (every snapshot point of it local to their owner, pcd_denoiser_set_coverage_spheres), four ranks
    sharing the GPU -- the band and the spheres priced for the run's drift, so no re-plan (round 5 allowed two, its
    spheres being snapshot-sized) -- and the one-GPU result within 1e-6 x bbox."""
    import torch.multiprocessing as mp
    pos, nrm = _cloud(gpu)
    d = _d(pos)
    out, cloud = str(tmp_path / "sph4.npz"), str(tmp_path / "cloud.npz")
    np.savez(cloud, pos=pos.cpu().numpy(), n=nrm.cpu().numpy())
    mp.spawn(_worker, args=(4, _free_port(), out, cloud, d, "gloo", False, None, 0.5), nprocs=4, join=True)
    res = np.load(out)
    report(f"coverage spheres: {int(res['spheres'])} spheres, halo rows on rank 0 {int(res['halo'])}, "
           f"replans {int(res['replans'])}")
    assert int(res["spheres"]) > 100 and int(res["replans"]) == 0
    rp, rn = _fused(pos, nrm, d)
    bbox = float(np.linalg.norm(rp.max(0) - rp.min(0)))
    np.testing.assert_allclose(res["pos"], rp, rtol=0, atol=1e-6 * bbox)
    np.testing.assert_allclose(res["n"], rn, rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_sphere_members_chunked_per_owner(gpu):
    """Spheres.around finds the members a bounded chunk of centres at a time and keeps one set per owner rank: the sets
    equal the brute-force members (every snapshot point within 1.0001 R of a centre, unioned per centre owner) at any
    chunk size."""
    from pcd_slab import Spheres, _cut
    pos, _ = _cloud(gpu)
    owner = _cut(pos, 4)[2]
    g = torch.Generator(device="cpu").manual_seed(3)
    ids = torch.randperm(pos.size(0), generator=g)[:300].to(gpu)
    radii = (0.01 + 0.03 * torch.rand(300, generator=g)).to(gpu)
    ref = {}
    for c, r in zip(ids.tolist(), radii.tolist()):
        d = (pos - pos[c]).norm(dim=1)
        m = torch.nonzero(d <= r * 1.0001).flatten()
        o = int(owner[c])
        ref[o] = torch.unique(torch.cat([ref.get(o, m[:0]), m]))
    for chunk in (500, 32_000_000):
        sp = Spheres.around(pos, ids, radii, owner, chunk_members=chunk)
        assert sorted(sp.by_rank) == sorted(ref)
        for o, m in ref.items():
            got = set(sp.by_rank[o].tolist())
            want = set(m.tolist())
            # (the library's radius test is fp32 on squared distances: rows on the 1.0001 R shell may differ)
            assert len(got ^ want) <= max(2, len(want) // 1000), (o, len(got ^ want))
