"""Normal voting tensors (drop-in for Pointcloud/Modules/Decompositionor.py, hot-path subset).

getBetterFilteredNVT -> pcd_nvt_csr: per segment, gather (v_j, n_j), threshold, accumulate the 6 unique entries of
T, Σw = 0 fallback, in-register 3x3 eigen-decomposition restating LAPACK ssyevd (ssytd2 + ssteqr, the signs MKL's
torch.linalg.eigh produces; reference Decompositionor.py:278-300).
Decomposition.getVUSmoothedNormals -> pcd_vu_smooth (:92-106); getNVTFeatures / getClasses -> pcd_classify (:57-69).
CPSD path: getNormalFilteredNVT -> pcd_nvt_normal_csr (:260-276), getNormalFilteredPVT -> pcd_pvt_normal_csr
(:172-211), Decomposition.getVUFeatures (:84-85).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

import pcd_native as _nat
from .Selector import Selection
from .Utils import GeneralUtils


@dataclass
class Decomposition:
    eigval: torch.Tensor   # (m, 3) ascending
    eigvec: torch.Tensor   # (m, 3, 3) columns

    def __post_init__(self):
        assert self.eigval.dim() == 2 and self.eigval.size(1) == 3 and self.eigval.is_floating_point()
        assert self.eigvec.dim() == 3 and self.eigvec.size(1) == 3 and self.eigvec.size(2) == 3
        assert self.eigvec.is_floating_point()
        assert self.eigval.size(0) == self.eigvec.size(0)

    def __len__(self):
        return self.eigval.size(0)

    def getNVTFeatures(self):
        """(planarity, linearity, sphericity) with λ1 ≥ λ2 ≥ λ3."""
        dev = self.eigval.device
        _, feat = _nat.classify(_nat.f32(self.eigval), 1.0, want_features=True)
        feat = feat.to(dev)
        return feat[:, 0], feat[:, 1], feat[:, 2]

    def getClasses(self, scale: float = 0.2) -> torch.Tensor:
        """argmax(scale·planarity, linearity, sphericity): 0 flat, 1 edge, 2 corner."""
        cls, _ = _nat.classify(_nat.f32(self.eigval), scale)
        return cls.to(self.eigval.device)

    def getVUFeatures(self, tau: float) -> torch.Tensor:
        """Decompositionor.py:84-85: number of eigenvalues below tau, mod 3."""
        return (self.eigval < tau).sum(dim=1) % 3

    def getVUSmoothedNormals(self, n: torch.Tensor, tau: float = 0.3, d: float = 3):
        """Decompositionor.py:92-106 as the reference writes it: f_n = normalize(d·n + Eᵀ·M·E·n), with E[r][k] the r-th
        component of the k-th eigenvector in descending eigenvalue order and M = diag([λ_(r) > τ]) indexed by that
        rank (NOT the projector Σ_k [λ_k > τ] (e_k·n) e_k = E·M·Eᵀ·n: the two agree only for M = 0 or I, so the
        result depends on LAPACK's eigenvector signs -- pcd_device.h vu_smooth)."""
        out = _nat.vu_smooth(_nat.f32(self.eigval), _nat.f32(self.eigvec), _nat.f32(n), tau, d)
        return out.to(n.device)


class Decompositionor:

    def __init__(self, graph):
        GeneralUtils.validateAttributes(graph, ["pos"])
        self.graph = graph

    def getBetterFilteredNVT(self, selection: Selection, _n: torch.Tensor, rho: float = 0.9) -> Decomposition:
        dev = self.graph.pos.device
        pos = _nat.f32(self.graph.pos)
        ev, evec = _nat.nvt_csr(pos, _nat.f32(_n), _nat.i64(selection.i), _nat.i64(selection.slices),
                                _nat.i64(selection.j), rho)
        return Decomposition(ev.to(dev), evec.to(dev))

    def getNormalFilteredNVT(self, selection: Selection, _n: torch.Tensor, rho: float = 0.9) -> Decomposition:
        """w_ij = acos(n_i . n_j) <= rho; T_i = Σ w n_j n_jᵀ / Σ w, n_i n_iᵀ where nothing votes."""
        dev = self.graph.pos.device
        ev, evec = _nat.nvt_normal_csr(_nat.f32(_n), _nat.i64(selection.i), _nat.i64(selection.slices),
                                       _nat.i64(selection.j), rho)
        return Decomposition(ev.to(dev), evec.to(dev))

    def getNormalFilteredPVT(self, selection: Selection, _n: torch.Tensor, rho: float = 0.9) -> Decomposition:
        """Weighted covariance of the voting neighbours about their weighted mean (all vote if none does)."""
        dev = self.graph.pos.device
        ev, evec = _nat.pvt_normal_csr(_nat.f32(self.graph.pos), _nat.f32(_n), _nat.i64(selection.i),
                                       _nat.i64(selection.slices), _nat.i64(selection.j), rho)
        return Decomposition(ev.to(dev), evec.to(dev))
