"""Mesh container + normal-guided vertex update (drop-in for PatchGeneration/Modules/Mesh.py, hot-path subset).

`updateVertices(n, k)` (reference Mesh.py:377-418, Vertex_updating.ipynb Algorithm 3) runs k Jacobi sweeps of
    v_i += Σ_{f∋i} Σ_{c∈f} n_f (n_f · (v_c − v_i)) / (3 deg_i)
in fp64 on the HIP device (pcd_mesh_update, one thread per vertex over the vertex->face CSR) and writes the result
back into `self.v` in place, like the reference's `v += scaled_S`.
The vertex-triangle adjacency is igl's format (VF = incident faces grouped by vertex in face order, NI = offsets)
computed here without igl.
"""
from __future__ import annotations

import numpy as np
import torch

import pcd_native as _nat


def vertex_triangle_adjacency(f: np.ndarray, nv: int):
    """igl.vertex_triangle_adjacency(f, nv) -> (VF, NI)."""
    flat = np.asarray(f, dtype=np.int64).reshape(-1)
    order = np.argsort(flat, kind="stable")
    vf = (order // 3).astype(np.int64)
    counts = np.bincount(flat, minlength=nv)
    ni = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return vf, ni


class Mesh:
    def __init__(self, v, f, noise_factor=0, f2f=None, vta=None, gt=None):
        self.v = v
        self.f = f
        self.noise_factor = noise_factor
        self.f2f = f2f
        self.vta = vta if vta is not None else vertex_triangle_adjacency(f, len(v))
        self.gt = gt

    @classmethod
    def readFile(cls, file_path: str) -> "Mesh":
        from Pointcloud.Modules.Object import read_obj_arrays
        v, _, f, _ = read_obj_arrays(file_path)
        return cls(v, f)

    def getVertices(self):
        return self.v

    def getFaceNormals(self):
        """Unit normals of (v1 − v0) × (v2 − v1) per face (Mesh.py:110-114)."""
        fvs = self.getVertices()[self.f]
        cr = np.cross(fvs[:, 1, :] - fvs[:, 0, :], fvs[:, 2, :] - fvs[:, 1, :])
        return cr / np.linalg.norm(cr, axis=1)[:, None]

    def getVertexTriangleAdjacency(self):
        return self.vta

    def updateVertices(self, n, k=15):
        v = self.getVertices()
        vf, ni = self.getVertexTriangleAdjacency()
        dev = _nat.device()
        vd = torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64)).to(dev)
        fd = torch.as_tensor(np.ascontiguousarray(self.f, dtype=np.int64)).to(dev)
        nd = torch.as_tensor(np.ascontiguousarray(n, dtype=np.float64)).to(dev)
        vfd = torch.as_tensor(np.ascontiguousarray(vf, dtype=np.int64)).to(dev)
        nid = torch.as_tensor(np.ascontiguousarray(ni, dtype=np.int64)).to(dev)
        assert nd.shape == fd.shape, "one normal per face"
        _nat.mesh_update(vd, fd, nd, vfd, nid, k)
        v[...] = vd.cpu().numpy().astype(v.dtype, copy=False)
