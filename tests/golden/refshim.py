"""In-container shims that let the *reference* Python hot path be imported for golden-vector generation.

TEST INFRASTRUCTURE ONLY.  Never imported by the product package, never shipped to the GPU box as a
dependency of anything that runs there.  Used exclusively by ``tests/golden/make_golden.py`` in the
build container, where ``/root/reference`` exists.

The reference (Ruubje/Normal-Guided-Pointcloud-Denoiser) imports third-party packages that are absent
here (SURVEY.md §8(c) "Shim contract").  Each shim below restates the published behaviour of the one
function the hot path calls:

* ``torch_geometric.data.Data``           attribute bag; num_nodes = pos.size(0), num_edges = edge_index.size(1)
* ``torch_geometric.utils.sort_edge_index`` lexicographic (row, col) sort
* ``torch_geometric.utils.to_undirected``  union of both directions, deduplicated (used by the MST only)
* ``torch_geometric.nn.pool.knn(x, y, k)``  for each y the k nearest x -> [2, |y|*k] (row0 = y, row1 = x)
* ``torch_scatter.scatter_{sum,mean,max}`` zero-initialised segment reductions (torch_scatter 2.0.9)
* ``torch_cluster.knn_graph(x, k, flow)``  k nearest excluding self; row0 = centre for "target_to_source"
* ``igl``, ``open3d``, ``robust_laplacian``, ``meshplot``, ``polyscope``: stubs that raise if called.
"""
from __future__ import annotations

import sys
import types

import numpy as np
import torch
from scipy.spatial import cKDTree


def _stub(name):
    def f(*a, **k):
        raise RuntimeError(f"shim: {name} is not available in this container")
    return f


class Data:
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def num_nodes(self):
        return self.pos.size(0)

    @property
    def num_edges(self):
        return self.edge_index.size(1)


def sort_edge_index(edge_index, edge_attr=None, num_nodes=None):
    n = int(edge_index.max()) + 1 if num_nodes is None else num_nodes
    key = edge_index[0] * n + edge_index[1]
    perm = torch.argsort(key, stable=True)
    out = edge_index[:, perm]
    if edge_attr is not None:
        return out, edge_attr[perm]
    return out


def to_undirected(edge_index, edge_attr=None, num_nodes=None, reduce="add"):
    n = int(edge_index.max()) + 1 if num_nodes is None else num_nodes
    ei = torch.cat([edge_index, edge_index.flip(0)], dim=1)
    key = ei[0] * n + ei[1]
    uniq, inv = torch.unique(key, return_inverse=True)
    out = torch.stack([uniq // n, uniq % n])
    if edge_attr is None:
        return out
    ea = torch.cat([edge_attr, edge_attr])
    red = torch.zeros(uniq.size(0), dtype=ea.dtype).index_add_(0, inv, ea)
    return out, red


def knn(x, y, k, batch_x=None, batch_y=None):
    tree = cKDTree(x.detach().cpu().double().numpy())
    _, idx = tree.query(y.detach().cpu().double().numpy(), k=k)
    idx = np.asarray(idx).reshape(y.size(0), k)
    row = np.repeat(np.arange(y.size(0)), k)
    return torch.stack([torch.from_numpy(row), torch.from_numpy(idx.reshape(-1))]).long()


def knn_graph(x, k, batch=None, loop=False, flow="source_to_target", **kw):
    pts = x.detach().cpu().double().numpy()
    tree = cKDTree(pts)
    _, idx = tree.query(pts, k=k + (0 if loop else 1))
    idx = np.asarray(idx).reshape(pts.shape[0], -1)
    if not loop:
        # drop the self column (column 0 unless duplicates precede it)
        n = pts.shape[0]
        out = np.empty((n, k), dtype=np.int64)
        for r in range(n):
            row = [c for c in idx[r] if c != r][:k]
            out[r] = row
        idx = out
    centre = torch.from_numpy(np.repeat(np.arange(pts.shape[0]), k))
    nbr = torch.from_numpy(idx.reshape(-1))
    if flow == "target_to_source":
        return torch.stack([centre, nbr]).long()
    return torch.stack([nbr, centre]).long()


def _scatter(src, index, dim=0, dim_size=None, reduce="sum"):
    assert dim == 0
    index = index.long()
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    shape = (dim_size,) + tuple(src.shape[1:])
    out = torch.zeros(shape, dtype=src.dtype)
    if reduce == "sum":
        return out.index_add_(0, index, src)
    if reduce == "mean":
        s = out.index_add_(0, index, src)
        c = torch.zeros(dim_size, dtype=src.dtype).index_add_(0, index, torch.ones(index.size(0), dtype=src.dtype))
        c = c.clamp(min=1).view((-1,) + (1,) * (src.dim() - 1))
        return s / c
    if reduce == "max":
        idx = index.view((-1,) + (1,) * (src.dim() - 1)).expand_as(src)
        return out.scatter_reduce_(0, idx, src, "amax", include_self=False), None
    raise ValueError(reduce)


def scatter_sum(src, index, dim=0, dim_size=None, out=None):
    return _scatter(src, index, dim, dim_size, "sum")


def scatter_mean(src, index, dim=0, dim_size=None, out=None):
    return _scatter(src, index, dim, dim_size, "mean")


def scatter_max(src, index, dim=0, dim_size=None, out=None):
    return _scatter(src, index, dim, dim_size, "max")


def degree(index, num_nodes=None, dtype=None):
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    return torch.zeros(n, dtype=dtype or torch.float).index_add_(0, index, torch.ones(index.size(0), dtype=dtype or torch.float))


class SamplePoints:
    def __init__(self, *a, **k):
        raise RuntimeError("shim: SamplePoints unavailable")


def install():
    """Register the shim modules in ``sys.modules`` (idempotent)."""
    if "torch_geometric" in sys.modules and getattr(sys.modules["torch_geometric"], "_is_shim", False):
        return

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m._is_shim = True
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    tg = mod("torch_geometric")
    tg.data = mod("torch_geometric.data", Data=Data)
    tg.utils = mod("torch_geometric.utils", sort_edge_index=sort_edge_index, to_undirected=to_undirected,
                   degree=degree, subgraph=_stub("subgraph"))
    tg.nn = mod("torch_geometric.nn")
    tg.nn.pool = mod("torch_geometric.nn.pool", knn=knn)
    tg.transforms = mod("torch_geometric.transforms", SamplePoints=SamplePoints)
    tg.loader = mod("torch_geometric.loader", DataLoader=_stub("DataLoader"))
    mod("torch_scatter", scatter_sum=scatter_sum, scatter_mean=scatter_mean, scatter_max=scatter_max)
    mod("torch_cluster", knn_graph=knn_graph)
    igl_names = ["vertex_triangle_adjacency", "per_vertex_normals", "per_face_normals", "barycenter",
                 "doublearea", "read_obj", "triangle_triangle_adjacency", "read_triangle_mesh", "write_obj"]
    mod("igl", **{n: _stub("igl." + n) for n in igl_names})
    o3d = mod("open3d")
    o3d.io = mod("open3d.io", read_point_cloud=_stub("open3d.io.read_point_cloud"))
    mod("robust_laplacian", point_cloud_laplacian=_stub("robust_laplacian.point_cloud_laplacian"))
    mod("meshplot", plot=_stub("meshplot.plot"), subplot=_stub("meshplot.subplot"))
    mod("polyscope", init=_stub("polyscope.init"))


def read_obj(path):
    """Minimal OBJ reader (v / f lines) – igl is absent."""
    v, f = [], []
    with open(path) as fh:
        for line in fh:
            if line.startswith("v "):
                v.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                f.append([int(t.split("/")[0]) - 1 for t in line.split()[1:4]])
    return np.asarray(v, dtype=np.float64), np.asarray(f, dtype=np.int64).reshape(-1, 3)
