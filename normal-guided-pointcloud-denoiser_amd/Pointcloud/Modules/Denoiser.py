"""Class-specific position updates (drop-in for Pointcloud/Modules/Denoiser.py).

Every step is one pcd_step_csr launch over the selection's segments: 3x3 accumulation in registers, then the
reference's torch.linalg.inv_ex restated operation for operation (MKL getrf(Aᵀ) + getrs('T'), pcd_device.h inv3_ref)
and its einsum-order product, with the exact-zero-pivot mask (inv_ex info) and the displacement clamp -- with the
reference's own inputs injected the edge / feature / corner steps are bit-identical to it
(tests/test_gpu_stages.py, test_capi.py::test_host_inv3_matches_torch_bitwise).  flat_step / new_step first
reduce the GLOBAL centre and spread of all neighbour rows (Denoiser.py:106-107, :138) on the device.
Reference lines: corner_step :26-51, edge_step :53-88, flat_step :90-119, new_step :121-172,
feature_step :174-219, dummy_step :221-232.
"""
from __future__ import annotations

import torch

import pcd_native as _nat
from .Selector import Selection


class Denoiser:
    def __init__(self, graph):
        assert hasattr(graph, "pos") and graph.pos is not None
        assert graph.pos.dim() == 2
        assert graph.pos.size(1) == 3
        self.graph = graph

    def _run(self, kind, selection: Selection, n: torch.Tensor, d: float, alpha: float, edge_vectors=None):
        _pos = self.graph.pos
        assert n.dim() == 2
        assert _pos.size(0) == n.size(0)
        assert n.size(1) == 3
        out = _nat.step_csr(kind, _nat.f32(_pos), _nat.f32(n),
                            None if edge_vectors is None else _nat.f32(edge_vectors),
                            _nat.i64(selection.i), _nat.i64(selection.slices), _nat.i64(selection.j),
                            float(d), float(alpha))
        return out.to(_pos.device)

    def corner_step(self, selection: Selection, n: torch.Tensor, d: float, alpha: float = 0.1):
        return self._run(_nat.STEP_CORNER, selection, n, d, alpha)

    def edge_step(self, selection: Selection, n: torch.Tensor, edge_vectors: torch.Tensor, d: float, alpha: float = 0.1):
        return self._run(_nat.STEP_EDGE, selection, n, d, alpha, edge_vectors)

    def flat_step(self, selection: Selection, n: torch.Tensor, d: float, alpha: float = 0.1):
        return self._run(_nat.STEP_FLAT, selection, n, d, alpha)

    def new_step(self, selection: Selection, n: torch.Tensor, d: float, alpha: float = 0.1):
        return self._run(_nat.STEP_NEW, selection, n, d, alpha)

    def feature_step(self, selection: Selection, n: torch.Tensor, d: float, alpha: float = 0.1):
        return self._run(_nat.STEP_FEATURE, selection, n, d, alpha)

    def dummy_step(self, selection: Selection, n: torch.Tensor, d: float, alpha: float = 0.1):
        _pos = self.graph.pos
        assert n.dim() == 2
        assert _pos.size(0) == n.size(0)
        assert n.size(1) == 3
        return _pos[selection.i.to(_pos.device)].clone()


# name of a bound step -> kernel kind (strategy dicts of denoiseUntilMinimumError, Processor.py:162-170)
STEP_KINDS = {"flat_step": _nat.STEP_FLAT, "edge_step": _nat.STEP_EDGE, "feature_step": _nat.STEP_FEATURE,
              "corner_step": _nat.STEP_CORNER, "new_step": _nat.STEP_NEW, "dummy_step": _nat.STEP_DUMMY}
