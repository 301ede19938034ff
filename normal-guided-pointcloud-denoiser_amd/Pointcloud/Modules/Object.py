"""Point-cloud container and OBJ I/O (drop-in for Pointcloud/Modules/Object.py:43-162, Pointcloud class).

The reference reads OBJ through igl; this reader parses `v`, `vn` and `f` records itself (igl is not a
dependency here).  `sampleObj` draws area-weighted barycentric samples with face normals (the reference uses
torch_geometric.transforms.SamplePoints) on the requested device.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from .Utils import TorchUtils


def read_obj_arrays(file_path: str):
    """(v float64 [V,3], vn float64 [Vn,3], fv int64 [F,3], fn int64 [F,3]) from an OBJ (triangles; polygons fanned)."""
    v, vn, fv, fn = [], [], [], []
    with open(file_path) as fh:
        for line in fh:
            if line.startswith("v "):
                v.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("vn "):
                vn.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                toks = line.split()[1:]
                vi = [int(t.split("/")[0]) for t in toks]
                ni = [int(t.split("/")[2]) if t.count("/") == 2 and t.split("/")[2] else 0 for t in toks]
                for a in range(1, len(vi) - 1):
                    tri = (vi[0], vi[a], vi[a + 1])
                    fv.append([x - 1 if x > 0 else len(v) + x for x in tri])
                    if all(ni):
                        tn = (ni[0], ni[a], ni[a + 1])
                        fn.append([x - 1 if x > 0 else len(vn) + x for x in tn])
    as_f = lambda a: np.asarray(a, dtype=np.float64).reshape(-1, 3)
    as_i = lambda a: np.asarray(a, dtype=np.int64).reshape(-1, 3)
    return as_f(v), as_f(vn), as_i(fv), as_i(fn) if len(fn) == len(fv) else np.zeros((0, 3), np.int64)


class Pointcloud:

    def __init__(self, v: torch.Tensor, n: torch.Tensor = None) -> None:
        assert v.is_floating_point()
        assert v.dim() == 2
        assert v.size(1) == 3
        if n is not None:
            assert n.is_floating_point()
            assert n.dim() == 2
            assert n.size(1) == 3
            assert v.size(0) == n.size(0)
        self.v = v
        self.n = n
        self.file_path = None

    def saveObj(self, file_path: str) -> None:
        with open(file_path, "x") as f:
            f.write("# pcd-mi355x\n")
            for row in self.v.tolist():
                f.write("v " + " ".join(str(x) for x in row) + "\n")
            if self.n is not None:
                for row in self.n.tolist():
                    f.write("vn " + " ".join(str(x) for x in row) + "\n")
        self.file_path = file_path

    @classmethod
    def loadObj(cls, file_path: str, device="cpu") -> "Pointcloud":
        path = Path(file_path)
        assert path.is_file()
        assert path.suffix == ".obj"
        v, n, fv, fn = read_obj_arrays(file_path)
        v = torch.tensor(v, dtype=torch.float32, device=device)
        n = torch.tensor(n, dtype=torch.float32, device=device)
        if n.size(0) > 0 and fn.shape[0] > 0:
            pc = Pointcloud(v, TorchUtils.face2vertexNormals(
                v, torch.tensor(fv, device=device), n, torch.tensor(fn, device=device)))
        elif n.size(0) > 0 and v.size(0) == n.size(0):
            pc = Pointcloud(v, n)
        else:
            pc = Pointcloud(v)
        pc.file_path = file_path
        return pc

    @classmethod
    def loadXYZ(cls, file_path: str, device="cpu") -> "Pointcloud":
        path = Path(file_path)
        assert path.is_file()
        assert path.suffix in (".xyz", ".clean_xyz")
        v = np.loadtxt(file_path, dtype=np.float64, ndmin=2)[:, :3]
        pc = Pointcloud(torch.tensor(v, dtype=torch.float32, device=device))
        pc.file_path = file_path
        return pc

    @classmethod
    def sampleObj(cls, file_path: str, num_points: int, device="cpu", generator: torch.Generator = None) -> "Pointcloud":
        """Area-weighted uniform samples of the mesh surface with the sampled face's unit normal."""
        path = Path(file_path)
        assert path.is_file()
        assert path.suffix == ".obj"
        v, _, fv, _ = read_obj_arrays(file_path)
        assert v.shape[1] == 3 and fv.shape[1] == 3
        # sampled where the cloud will live (the 10M / 80M bench clouds are drawn on the GPU, never through host RAM)
        pos, nrm = sample_surface(torch.tensor(v, dtype=torch.float32, device=device),
                                  torch.tensor(fv, device=device), num_points, generator=generator)
        pc = Pointcloud(pos, nrm)
        pc.file_path = file_path
        return pc

    def hasNormals(self):
        return self.n is not None

    def hasFilePath(self):
        return self.file_path is not None


def sample_surface(v: torch.Tensor, f: torch.Tensor, num: int, generator: torch.Generator = None,
                   return_faces: bool = False):
    """Area-weighted barycentric sampling (the SamplePoints transform's algorithm) -> (pos, face normals[, face ids]).
    Faces are drawn by inversion of the area CDF (float64, scanned on the host) with uniform draws from `generator`:
    the same distribution as SamplePoints' torch.multinomial, but the same seed gives the same cloud on every call and
    device (a device multinomial is not bitwise reproducible between calls, so two processes drawing the bench's
    cloud would hold different clouds)."""
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    cr = torch.cross(b - a, c - a, dim=1)
    area = cr.norm(dim=1)
    fn = cr / area.clamp(min=1e-30)[:, None]
    dev = generator.device if generator is not None else v.device
    cdf = torch.cumsum(area.double().cpu(), 0)
    u = torch.rand(num, generator=generator, device=dev, dtype=torch.float64) * cdf[-1].item()
    fid = torch.searchsorted(cdf.to(dev), u).clamp_(max=len(cdf) - 1).to(v.device)
    uv = torch.rand((num, 2), generator=generator, device=dev).to(v.device)
    flip = uv.sum(1) > 1
    uv[flip] = 1 - uv[flip]
    pos = a[fid] + uv[:, :1] * (b[fid] - a[fid]) + uv[:, 1:] * (c[fid] - a[fid])
    return (pos, fn[fid], fid) if return_faces else (pos, fn[fid])
