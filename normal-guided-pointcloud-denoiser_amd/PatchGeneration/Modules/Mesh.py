"""Mesh container + normal-guided vertex update (drop-in for PatchGeneration/Modules/Mesh.py, hot-path subset).

`updateVertices(n, k)` (reference Mesh.py:377-418, Vertex_updating.ipynb Algorithm 3) runs k Jacobi sweeps of
    v_i += Σ_{f∋i} Σ_{c∈f} n_f (n_f · (v_c − v_i)) / (3 deg_i)
in fp64 on the HIP device (pcd_mesh_update, one thread per vertex over the vertex->face CSR) and writes the result
back into `self.v` in place, like the reference's `v += scaled_S`.
The vertex-triangle adjacency is igl's format (VF = incident faces grouped by vertex in face order, NI = offsets),
built on the device (pcd_mesh_vta: a stable radix sort of the corners by vertex) and kept there with the faces;
`updateVertices(n, k, fp32=True)` runs the fp32 kernel (pcd_mesh_update_f32).
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
        self._topo = {}           # device copies of the faces and the adjacency, per precision
        self.v = v
        self.f = f
        self.noise_factor = noise_factor
        self.f2f = f2f
        self.vta = vta            # igl (VF, NI); None: built on the device on first use (pcd_mesh_vta)
        self.gt = gt

    # assigning the faces or the adjacency drops the device copies built from them
    @property
    def f(self):
        return self._f

    @f.setter
    def f(self, value):
        self._f = value
        self._topo = {}

    @property
    def vta(self):
        return self._vta

    @vta.setter
    def vta(self, value):
        self._vta = value
        self._topo = {}

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
        if self.vta is None:
            vf, ni = self._topology(False)[1:]
            self._vta = (vf.cpu().numpy(), ni.cpu().numpy())   # (the device copies it came from stay valid)
        return self.vta

    def _topology(self, fp32: bool):
        """(faces, VF, NI) on the device, int32 for the fp32 path, int64 for fp64; the adjacency is the caller's vta
        when one was given, else built on the device.  Cached per precision together with a host copy of the faces
        it was built from: an in-place edit of self.f (same object, new contents) rebuilds it."""
        key = bool(fp32)
        hit = self._topo.get(key)
        if hit is not None and not np.array_equal(hit[0], self.f):
            hit = None
        if hit is None:
            it = torch.int32 if fp32 else torch.int64
            f_host = np.array(self.f, copy=True)
            fd = torch.as_tensor(np.ascontiguousarray(f_host)).to(_nat.device()).to(it).contiguous()
            if self.vta is not None:
                vf, ni = (torch.as_tensor(np.ascontiguousarray(a)).to(fd.device).to(it) for a in self.vta)
            else:
                vf, ni = _nat.mesh_vta(fd, len(self.v), out_dtype=it)
            hit = (f_host, fd, vf.contiguous(), ni.contiguous())
            self._topo[key] = hit
        return hit[1:]

    def updateVertices(self, n, k=15, fp32: bool = False):
        """Mesh.py:377-418: k Jacobi sweeps, in place on self.v.  fp32=True runs the fp32 kernel (float4 rows, int32
        topology) instead of the reference's fp64 arithmetic."""
        v = self.getVertices()
        fd, vfd, nid = self._topology(fp32)
        dev = fd.device
        dt = torch.float32 if fp32 else torch.float64
        vd = torch.as_tensor(np.ascontiguousarray(v)).to(dev).to(dt).contiguous()
        nd = torch.as_tensor(np.ascontiguousarray(n)).to(dev).to(dt).contiguous()
        assert nd.shape == fd.shape, "one normal per face"
        if fp32:
            _nat.mesh_update_f32(vd, fd, nd, vfd, nid, k)
        else:
            _nat.mesh_update(vd, fd, nd, vfd, nid, k)
        v[...] = vd.cpu().numpy().astype(v.dtype, copy=False)
