"""GPU normal orientation: pcd_orient_normals_mst_gpu against the host Kruskal + DFS
pcd_orient_normals_mst (itself checked against the oracle and the reference's oriented lattice normals in
test_capi.py / test_oracle_golden.py).  The bar is bit-exact: orientation is a sign per point, and the device
MST is the same unique forest under (cost, edge index) keys.
"""
import numpy as np
import pytest
import torch

import pcd_native as nat
from oracle import pcd_oracle as O
from Pointcloud.Modules.GraphBuilder import GraphBuilder
from Pointcloud.Modules.Object import Pointcloud

pytestmark = pytest.mark.gpu


def host_orient(pos, n, a, b):
    n = n.detach().cpu().float().contiguous().clone()
    nat.orient_normals_mst(pos.detach().cpu().float().contiguous(), n, a.detach().cpu().long().contiguous(),
                           b.detach().cpu().long().contiguous())
    return n


def both(pos, n, a, b, gpu):
    ref = host_orient(pos, n, a, b)
    out = nat.orient_normals_mst_gpu(pos.to(gpu), n.to(gpu), a.to(gpu), b.to(gpu)).cpu()
    return out, ref


def knn_edges(pos, k, gpu):
    gb = GraphBuilder(Pointcloud(pos.to(gpu).clone()))
    ei = gb.getKNNEdgeIndex(k)
    return ei[0], ei[1]


def pca_normals(pos, a, b, k, gpu):
    gb = GraphBuilder(Pointcloud(pos.to(gpu).clone()))
    return gb.getPVTDecompositionWithKNN(torch.stack([a, b]).to(gpu))[..., 0]


def test_fandisk_bitwise(golden, gpu):
    fan = golden("fandisk_k32")
    pos = torch.from_numpy(fan["pos0"]).float()
    a, b = knn_edges(pos, 12, gpu)
    n = pca_normals(pos, a, b, 12, gpu)
    out, ref = both(pos, n, a, b, gpu)
    assert torch.equal(out, ref)
    # the reference's own oriented normals for this input
    assert ((out.numpy() * fan["n0"]).sum(1) > 0.999).mean() > 0.99


def test_lattice_against_oracle(golden, gpu):
    lat = golden("lattice")
    pos = lat["n17_j1_pos"]
    nbr = O.knn_graph_noself(pos, 12)
    n0 = O.pca_normals_unoriented(pos, nbr).astype(np.float32)
    ref = O.orient_normals_mst(pos, n0.copy(), nbr)
    a = torch.from_numpy(np.repeat(np.arange(len(pos)), 12))
    b = torch.from_numpy(nbr.reshape(-1).copy())
    out = nat.orient_normals_mst_gpu(torch.from_numpy(pos).to(gpu), torch.from_numpy(n0).to(gpu), a.to(gpu),
                                     b.to(gpu)).cpu().numpy()
    assert ((out * ref).sum(1) > 0.999).mean() > 0.995
    assert (np.sign((out * lat["n17_j1_n"]).sum(1)) > 0).mean() > 0.99


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_surfaces_bitwise(seed, gpu):
    g = torch.Generator().manual_seed(seed)
    m = 20000
    uv = torch.rand(m, 2, generator=g) * 4 - 2
    z = torch.sin(uv[:, 0] * 2) * torch.cos(uv[:, 1] * 3) * 0.4
    pos = torch.cat([uv, z[:, None]], 1) + 0.002 * torch.randn(m, 3, generator=g)
    a, b = knn_edges(pos, 12, gpu)
    n = pca_normals(pos, a, b, 12, gpu).cpu()
    n = n * torch.where(torch.rand(m, 1, generator=g) < 0.5, -1.0, 1.0)
    out, ref = both(pos, n, a, b, gpu)
    assert torch.equal(out, ref)


def test_disconnected_components_untouched(gpu):
    # three far-apart clusters with kNN inside each: only the highest cluster's tree is oriented
    g = torch.Generator().manual_seed(7)
    parts = [torch.randn(3000, 3, generator=g) * torch.tensor([1.0, 1.0, 0.05]) + torch.tensor(c)
             for c in ([0.0, 0.0, 0.0], [100.0, 0.0, 5.0], [0.0, 100.0, -5.0])]
    pos = torch.cat(parts)
    a, b = knn_edges(pos, 10, gpu)
    n = torch.nn.functional.normalize(torch.randn(len(pos), 3, generator=g), dim=1)
    out, ref = both(pos, n, a, b, gpu)
    assert torch.equal(out, ref)
    assert torch.equal(out[:3000], n[:3000]) and torch.equal(out[6000:], n[6000:])


def test_ties_duplicates_self_edges(gpu):
    # quantised normals -> many equal costs (tie order = edge order), plus duplicated, reversed and self edges
    g = torch.Generator().manual_seed(3)
    m = 5000
    pos = torch.rand(m, 3, generator=g)
    n = torch.randint(-2, 3, (m, 3), generator=g).float()
    n[(n == 0).all(1)] = torch.tensor([0.0, 0.0, 1.0])
    n = torch.nn.functional.normalize(n, dim=1)
    a, b = knn_edges(pos, 8, gpu)
    a, b = a.cpu(), b.cpu()
    extra = torch.randint(0, m, (4000,), generator=g)
    a2 = torch.cat([a, b[:3000], extra, a[:2000]])
    b2 = torch.cat([b, a[:3000], extra, b[:2000]])
    perm = torch.randperm(len(a2), generator=g)
    out, ref = both(pos, n, a2[perm], b2[perm], gpu)
    assert torch.equal(out, ref)


def test_no_edges_and_tiny(gpu):
    pos = torch.tensor([[0.0, 0.0, 1.0], [0.0, 0.0, 2.0], [1.0, 0.0, 0.0]])
    n = torch.tensor([[0.0, 0.0, 1.0], [0.0, 0.6, -0.8], [1.0, 0.0, 0.0]])
    e = torch.zeros(0, dtype=torch.int64)
    out, ref = both(pos, n, e, e, gpu)
    assert torch.equal(out, ref)
    assert torch.equal(out[1], torch.tensor([0.0, -0.6, 0.8]))           # only the root is flipped up
    out, ref = both(pos, n, torch.tensor([1, 2]), torch.tensor([0, 1]), gpu)
    assert torch.equal(out, ref)


def test_bad_edge_rejected(gpu):
    pos = torch.rand(10, 3, device=gpu)
    n = torch.rand(10, 3, device=gpu)
    with pytest.raises(ValueError):
        nat.orient_normals_mst_gpu(pos, n, torch.tensor([0, 1], device=gpu), torch.tensor([1, 10], device=gpu))


def test_large_bitwise(gpu):
    # 400k points, 4.8M edges: deep trees (long Euler tours, many pointer-jumping rounds)
    g = torch.Generator().manual_seed(11)
    m = 400_000
    t = torch.rand(m, generator=g) * 40
    pos = torch.stack([torch.cos(t) * (1 + 0.1 * t), torch.sin(t) * (1 + 0.1 * t), torch.rand(m, generator=g)], 1)
    a, b = knn_edges(pos, 12, gpu)
    n = pca_normals(pos, a, b, 12, gpu).cpu()
    out, ref = both(pos, n, a, b, gpu)
    assert torch.equal(out, ref)
