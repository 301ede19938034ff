"""Neighbourhood selection (drop-in for Pointcloud/Modules/Selector.py, hot-path subset).

`Selector.__init__` freezes a snapshot of the positions it is given (the reference builds
scipy KDTree(graph.pos) once, Selector.py:138-141); `getKNNSelection` queries the CURRENT graph.pos against that
frozen snapshot (Selector.py:235-246).  Both run on the HIP device through libpcd (pcd_grid_build / pcd_knn).
`Selection` keeps the reference's CSR container contract (i, j, slices; Selector.py:41-134); its methods are
index plumbing on whatever device the tensors live on.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import pcd_native as _nat
from .Utils import GeneralUtils, TorchUtils


@dataclass
class Selection:
    i: torch.Tensor
    j: torch.Tensor
    slices: torch.Tensor

    def __len__(self):
        return self.slices.size(0) - 1

    def __getitem__(self, key: int):
        assert key >= 0 and key <= len(self)
        return self.j[self.slices[key]:self.slices[key + 1]]

    def __setattr__(self, name, value):
        if name == "i":
            self._assertI(value)
        if name == "j":
            self._assertJ(value)
        elif name == "slices":
            self._assertSlices(value)
        object.__setattr__(self, name, value)

    def _assertI(self, _i):
        assert _i.dim() == 1, f"Actual size of i: {_i.size()}"
        assert not _i.is_floating_point()
        if hasattr(self, "slices"):
            assert _i.size(0) == len(self)

    def _assertJ(self, _j):
        assert _j.dim() == 1, f"Actual size of data: {_j.size()}"
        assert not _j.is_floating_point()
        if hasattr(self, "slices"):
            assert _j.size(0) == self.slices[-1]

    def _assertSlices(self, _slices):
        assert _slices.dim() == 1
        assert not _slices.is_floating_point()
        assert _slices[0] == 0, f"Slider start: {_slices[0]}"
        if hasattr(self, "i"):
            assert self.i.size(0) == _slices.size(0) - 1
        if hasattr(self, "j"):
            assert self.j.size(0) == _slices[-1], f"Data size: {self.j.size(0)}\nSlices last entry: {_slices[-1]}"

    # dense kNN selections (slices = arange * k) are the common case; keep them dense through filter()
    def _dense_k(self):
        k = getattr(self, "_k", None)
        return k

    def filter(self, indices: torch.Tensor) -> "Selection":
        """Keep the segments at `indices` (positions into i), in that order (reference Selector.py:85-92)."""
        indices = indices.to(self.i.device)
        k = self._dense_k()
        new_i = self.i[indices]
        if k is not None:
            new_j = self.j.view(-1, k)[indices].reshape(-1)
            out = Selection(new_i, new_j, torch.arange(indices.numel() + 1, device=self.j.device) * k)
            object.__setattr__(out, "_k", k)
            return out
        starts = self.slices[indices]
        ends = self.slices[indices + 1]
        new_j = self.j[TorchUtils.rangeBoundariesToIndices(starts, ends)]
        new_slices = torch.cat([torch.zeros(1, dtype=ends.dtype, device=ends.device), (ends - starts).cumsum(0)])
        return Selection(new_i, new_j, new_slices)

    @classmethod
    def fromEdgeIndex(cls, edge_index: torch.Tensor) -> "Selection":
        n = int(edge_index.max()) + 1 if edge_index.numel() else 0
        order = torch.argsort(edge_index[0] * max(n, 1) + edge_index[1], stable=True)
        ei = edge_index[:, order]
        unique, counts = ei[0].unique(return_counts=True)
        slices = torch.zeros(unique.size(0) + 1, dtype=torch.long, device=ei.device)
        slices[1:] = counts.cumsum(0)
        return Selection(unique, ei[1].contiguous(), slices)

    def getEdgeIndex(self) -> torch.Tensor:
        _slices = self.slices
        assert _slices.dim() == 1, "slices must have 2 dimensions"
        assert not _slices.is_floating_point(), "slices must contain integers"
        starts, ends = _slices[:-1], _slices[1:]
        start = torch.repeat_interleave(self.i, ends - starts)
        end = self.j[TorchUtils.rangeBoundariesToIndices(starts, ends)]
        return torch.vstack([start[None], end[None]])

    def getBatchIndex(self) -> torch.Tensor:
        n = self.i.size(0)
        seg = torch.arange(n, device=self.slices.device)
        return torch.repeat_interleave(seg, self.slices[1:] - self.slices[:-1])

    def scatter(self, source: torch.Tensor, reduce: str) -> torch.Tensor:
        """Segment reduction of per-row values (torch_scatter sum / max / mean semantics)."""
        b = self.getBatchIndex().to(source.device)
        m = len(self)
        shape = (m,) + tuple(source.shape[1:])
        if reduce == "add":
            return torch.zeros(shape, dtype=source.dtype, device=source.device).index_add_(0, b, source)
        if reduce == "mean":
            s = torch.zeros(shape, dtype=source.dtype, device=source.device).index_add_(0, b, source)
            c = torch.bincount(b, minlength=m).clamp(min=1).to(source.dtype)
            return s / c.view((-1,) + (1,) * (source.dim() - 1))
        if reduce == "max":
            idx = b.view((-1,) + (1,) * (source.dim() - 1)).expand_as(source)
            out = torch.zeros(shape, dtype=source.dtype, device=source.device)
            return out.scatter_reduce_(0, idx, source, "amax", include_self=False), None
        raise ValueError(f"unknown reduce {reduce}")


class Selector:

    def __init__(self, graph, k_hint: int = 16):
        GeneralUtils.validateAttributes(graph, ["pos"])
        self.graph = graph
        # frozen snapshot of the positions at construction (never rebuilt), like scipy KDTree(graph.pos)
        self.grid = _nat.Grid(graph.pos, k_hint=k_hint)

    def getPointsInRangeSelectionVectorized(self, radii: torch.Tensor, indices: torch.Tensor = None) -> Selection:
        """Selector.py:214-230: every frozen-snapshot point within radii[r] of the r-th query (current position of
        indices[r], or of point r), ascending index -- scipy query_ball_point, here pcd_radius_count/_fill."""
        TorchUtils.validateIndices(indices)
        _graph = self.graph
        N = _graph.num_nodes if indices is None else indices.size(0)
        device = radii.device
        assert radii.dim() == 1
        assert radii.size(0) == N, f"Actual: {radii.size(0)}\nExpected: {N}"
        assert radii.is_floating_point()
        _pos = _graph.pos if indices is None else _graph.pos[indices]
        slices, j = self.grid.radius(_pos, radii.to(torch.float32))
        i = indices if indices is not None else torch.arange(N)
        return Selection(i.to(device), j.to(device), slices.to(device))

    def getPointsInRangeSelection(self, radius: float, indices: torch.Tensor = None) -> Selection:
        """Selector.py:232-233 (radius as a torch.float tensor over all points, as the reference builds it)."""
        return self.getPointsInRangeSelectionVectorized(
            torch.full((self.graph.num_nodes,), radius, dtype=torch.float, device=self.graph.pos.device), indices)

    def getKNNSelection(self, k: int, indices: torch.Tensor = None) -> Selection:
        _pos = self.graph.pos
        dev = _pos.device
        if indices is None:
            indices = torch.arange(_pos.size(0), dtype=torch.long, device=dev)
        if not torch.is_tensor(indices) or indices.is_floating_point():
            raise ValueError("indices should contain integer values and not floating point values.")
        q = _pos[indices.to(dev)]
        knn = self.grid.knn(q, k).to(dev)
        sel = Selection(indices.to(dev), knn.reshape(-1), torch.arange(knn.size(0) + 1, device=dev, dtype=torch.long) * k)
        object.__setattr__(sel, "_k", k)
        return sel
