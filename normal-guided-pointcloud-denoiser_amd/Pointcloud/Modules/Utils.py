"""Metrics and index plumbing (drop-in for Pointcloud/Modules/Utils.py, hot-path subset).

Kernels: averageEdgeLength -> pcd_edge_length_sum; Chamfer/Hausdorff/PaperDistance -> pcd_nn_dist over a
transient grid (kNN-1), replacing torch_geometric.nn.pool.knn (reference Utils.py:253-295).
Results come back on the device of the first input.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Collection

import torch

import pcd_native as _nat


class GeneralUtils:

    @classmethod
    def validateAttributes(cls, obj: Any, attrs: Collection[str]) -> None:
        """Reference Utils.py:56-66: raise ValueError if an attribute is missing or None."""
        for attr in attrs:
            if not hasattr(obj, attr) or getattr(obj, attr) is None:
                raise ValueError(f"Object does not have attribute '{attr}'.")


@dataclass
class SlicedTorchData:
    """CSR payload (data, slices) -- reference Utils.py:123-192 (container only)."""
    data: torch.Tensor
    slices: torch.Tensor

    def __len__(self):
        return self.slices.size(0) - 1

    def __getitem__(self, key: int):
        return self.data[self.slices[key]:self.slices[key + 1]]


def _nn(ref: torch.Tensor, q: torch.Tensor):
    """For every row of q: (squared distance, index) of its nearest row of ref (pcd_nn_dist).  The grid is sized for
    ~16 points a cell: the queries of an error metric (a noisy or denoised cloud against its surface) sit several point
    spacings off ref, and coarser cells reach them in fewer probes (10M points: 42 ms against 276 ms with ~1 point a
    cell, tools/nn_probe.py); the result is exact either way."""
    grid = _nat.Grid(ref, k_hint=32)
    return grid.nn(q)


class TorchUtils:

    @classmethod
    def validateIndices(cls, indices: torch.Tensor) -> None:
        assert indices is None or (not indices.is_floating_point() and indices.dim() == 1), \
            f"indices dimensions: {indices.dim()}\nindices type: {indices.dtype}"

    @classmethod
    def validateEdgeIndex(cls, _edge_index: torch.Tensor) -> None:
        assert not _edge_index.is_floating_point(), "_edge_index should be indices and not floating points.."
        assert _edge_index.dim() == 2, f"_edge_index dimensions: {_edge_index.dim()}"
        assert _edge_index.size(0) == 2, f"_edge_index first dimension: {_edge_index.size(0)}"

    @classmethod
    def validateKNNEdgeIndex(cls, _edge_index: torch.Tensor):
        """Every source node must have the same out-degree k; returns k (reference Utils.py:217-222)."""
        cls.validateEdgeIndex(_edge_index)
        counts = torch.bincount(_edge_index[0]).unique()
        counts = counts[counts > 0]
        assert counts.size(0) == 1
        return int(counts[0])

    @classmethod
    def face2vertexNormals(cls, v, fv, n, fn):
        assert v.dim() == 2 and fv.dim() == 2 and n.dim() == 2 and fn.dim() == 2
        assert v.is_floating_point() and n.is_floating_point() and not fv.is_floating_point() and not fn.is_floating_point()
        assert fv.size(0) == fn.size(0)
        assert v.size(1) == n.size(1)
        vn = torch.zeros_like(v)
        vn.index_add_(0, fv.reshape(-1), n[fn].reshape(-1, 3))
        return torch.nn.functional.normalize(vn, dim=-1)

    @classmethod
    def ChamferDistance(cls, pos0: torch.Tensor, pos1: torch.Tensor) -> torch.Tensor:
        """cat(||pos0[nn0(pos1)] - pos1||² (len |pos1|), ||pos1[nn1(pos0)] - pos0||² (len |pos0|))."""
        assert pos0.dim() == 2 and pos1.dim() == 2 and pos0.size(1) == 3 and pos1.size(1) == 3
        c0, _ = _nn(pos0, pos1)
        c1, _ = _nn(pos1, pos0)
        return torch.cat([c0, c1], dim=0).to(pos0.device)

    @classmethod
    def SingleChamferDistance(cls, pos0: torch.Tensor, pos1: torch.Tensor) -> torch.Tensor:
        """sCD: the first half of ChamferDistance, ||pos0[nn0(pos1)] - pos1||² for every point of pos1 (len |pos1|).
        With the reference's call order error_func(gt, denoised) (Processor.py:154,165, PostProcessing.ipynb:1024) this
        is the denoised -> ground-truth term.  The reference notebook calls TorchUtils.SingleChamferDistance, which its
        Utils.py does not define; this is that half of Utils.py:253-265."""
        assert pos0.dim() == 2 and pos1.dim() == 2 and pos0.size(1) == 3 and pos1.size(1) == 3
        c0, _ = _nn(pos0, pos1)
        return c0.to(pos0.device)

    @classmethod
    def HausdorffDistance(cls, pos0: torch.Tensor, pos1: torch.Tensor) -> torch.Tensor:
        assert pos0.dim() == 2 and pos1.dim() == 2 and pos0.size(1) == 3 and pos1.size(1) == 3
        c0, _ = _nn(pos0, pos1)
        c1, _ = _nn(pos1, pos0)
        return torch.cat([c0, c1], dim=0).sqrt().to(pos0.device)

    @classmethod
    def PaperDistance(cls, gt: torch.Tensor, noisy: torch.Tensor) -> torch.Tensor:
        """||gt[nn(noisy)] - noisy|| / bbox_diag(gt) per noisy point (reference Utils.py:281-295)."""
        assert gt.dim() == 2 and noisy.dim() == 2 and gt.size(1) == 3 and noisy.size(1) == 3
        g = _nat.f32(gt)
        diag = (g.max(dim=0).values - g.min(dim=0).values).norm(dim=0)
        d2, _ = _nn(g, noisy)
        return (d2.sqrt() / diag).to(noisy.device)

    @classmethod
    def averageEdgeLength(cls, pos: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        """mean_e ||pos[b_e] - pos[a_e]|| as a 0-dim fp32 tensor on pos.device (reference Utils.py:297-299)."""
        p = _nat.f32(pos)
        ei = _nat.i64(edge_index)
        e = ei.size(1)
        s = _nat.edge_length_sum(p, ei[0].contiguous(), ei[1].contiguous())
        return (s[0] / max(e, 1)).to(torch.float32).to(pos.device)

    @classmethod
    def pointcloudRadius(cls, pos: torch.Tensor):
        return (pos - pos.mean(dim=0, keepdim=True)).norm(dim=1).max(dim=0).values

    @classmethod
    def rangeBoundariesToIndices(cls, starts: torch.Tensor, ends: torch.Tensor) -> torch.Tensor:
        """Concatenate the ranges [starts[r], ends[r]) (empty / reversed ranges are dropped)."""
        assert starts.dtype == torch.long
        lens = ends - starts
        keep = lens > 0
        if not bool(keep.all()):
            starts, ends, lens = starts[keep], ends[keep], lens[keep]
        if lens.numel() == 0:
            return torch.empty(0, dtype=torch.long, device=starts.device)
        seg = torch.repeat_interleave(torch.arange(lens.numel(), device=starts.device), lens)
        first = torch.cumsum(lens, 0) - lens
        return starts[seg] + (torch.arange(seg.numel(), device=starts.device) - first[seg])
