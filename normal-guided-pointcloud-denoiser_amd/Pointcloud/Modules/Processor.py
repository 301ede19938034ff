"""Orchestrator (drop-in for Pointcloud/Modules/Processor.py, hot-path subset).

`denoise()` / `denoiseUntilMinimumError()` run the loop body of the reference (Processor.py:119-185) as the fused
libpcd loop (pcd_denoiser_*): kNN+NVT1+smoothing, NVT2+classes, then the class phases Gauss-Seidel in order, all on
device buffers in spatial order; results are written back into the caller's tensors with the reference's aliasing
(graph.pos mutated in place, graph.n rebound to f_n).  `getMyFeatureDecomposition()` keeps the op-by-op path
(Selector -> Decompositionor) because it must return the full Decomposition.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

import pcd_native as _nat
from .Decompositionor import Decompositionor
from .Denoiser import STEP_KINDS, Denoiser
from .GraphBuilder import GraphBuilder
from .Noise import Noise
from .Object import Pointcloud
from .Selector import Selector
from .Utils import GeneralUtils, TorchUtils

DEFAULT_ANGLE = math.pi * 5 / 12     # Processor.py:111
DEFAULT_ALPHAS = (1.0, 0.2, 1.0)     # Processor.py:122


class Processor:
    def __init__(self, pointcloud: Pointcloud, k_hint: int = 16):
        self.pointcloud = pointcloud
        self.graphBuilder = GraphBuilder(pointcloud)
        _graph = self.graphBuilder.graph
        self.graph = _graph
        self.selector = Selector(_graph, k_hint=k_hint)
        self.noise = Noise(_graph)
        self.denoiser = Denoiser(_graph)
        self.decompositionor = Decompositionor(_graph)
        self._fused = None

    # ------------------------------------------------------------------ op-by-op feature decomposition
    def getMyFeatureDecomposition(self, N: int = 2 ** 4, angle: float = None):
        angle = angle if angle is not None else DEFAULT_ANGLE
        n = self.graph.n
        selection = self.selector.getKNNSelection(N)
        nvt = self.decompositionor.getBetterFilteredNVT(selection, n, angle)
        filtered_normals = nvt.getVUSmoothedNormals(n)
        decomposition = self.decompositionor.getBetterFilteredNVT(selection, filtered_normals, angle)
        return decomposition, filtered_normals

    # ------------------------------------------------------------------ CPSD ("Martin") feature path
    def getMartinFeatureDecomposition(self, r: float, rho: float = 0.9):
        """Processor.py:102-108: radius selection -> normal-filtered NVT -> VU smoothing -> normal-filtered PVT."""
        _n = self.graph.n
        selection = self.selector.getPointsInRangeSelection(r)
        nvt = self.decompositionor.getNormalFilteredNVT(selection, _n, rho)
        filtered_normals = nvt.getVUSmoothedNormals(_n)
        decomposition = self.decompositionor.getNormalFilteredPVT(selection, filtered_normals, rho)
        return decomposition, filtered_normals

    def getVUDecomposition(self):
        """Processor.py:83-100: r = 2 x the mean kNN(6) graph edge length, rho = 0.95 for both votes."""
        _graph = self.graph
        _graph.edge_index = self.graphBuilder.getKNNEdgeIndex(6)
        mean_graph_edge_length = TorchUtils.averageEdgeLength(_graph.pos, _graph.edge_index)
        r = 2 * mean_graph_edge_length
        selection = self.selector.getPointsInRangeSelection(float(r))
        decompositionNVT = self.decompositionor.getNormalFilteredNVT(selection, _graph.n, rho=0.95)
        filtered_normals = decompositionNVT.getVUSmoothedNormals(_graph.n, tau=0.3, d=3)
        return self.decompositionor.getNormalFilteredPVT(selection, filtered_normals, rho=0.95)

    # ------------------------------------------------------------------ fused loop
    def _fused_for(self, k_max: int) -> _nat.FusedDenoiser:
        if self._fused is None or self._fused.k_max < k_max:
            # the same frozen snapshot, indexed with cells of about one list cap of points (pcd_native.fused_k_hint)
            grid = self.selector.grid
            kh = _nat.fused_k_hint(k_max)
            if kh and grid.k_hint != kh:
                grid = grid.rebuild(kh)
            self._fused = _nat.FusedDenoiser(grid, k_max)
        return self._fused

    def meanEdgeLength(self) -> torch.Tensor:
        """l of Processor.py:120 (kNN(6) rows, self row included)."""
        return TorchUtils.averageEdgeLength(self.graph.pos, self.selector.getKNNSelection(6).getEdgeIndex())

    def _run_fused(self, iterations: int, k: int, k_update: int, d: float, phases, angle=None,
                   return_classes: bool = False):
        g = self.graph
        GeneralUtils.validateAttributes(g, ["pos", "n"])
        fused = self._fused_for(max(k, k_update))
        fused.load(g.pos, g.n)
        params = _nat.make_params(k=k, k_update=k_update, rho=angle, d=float(d), phases=phases)
        fused.iterate(params, iterations)
        dev = _nat.device()
        pos_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
        n_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
        cls = torch.empty(g.num_nodes, dtype=torch.int64, device=dev) if return_classes else None
        fused.store(pos_out, n_out, cls)
        with torch.no_grad():
            g.pos.copy_(pos_out.to(g.pos.dtype))          # in place: keeps pointcloud.v aliased
        g.n = n_out.to(device=g.pos.device, dtype=g.pos.dtype)
        return cls

    def denoise(self, iterations: int = 2, k: int = 2 ** 4, k_update: int = 8, alphas=DEFAULT_ALPHAS,
                d: float = None, angle: float = None):
        """Processor.py:119-139.  Defaults reproduce the reference exactly (k=16, k_u=8, 2 iterations, d=2l)."""
        if d is None:
            d = 2 * float(self.meanEdgeLength())
        phases = ((0, _nat.STEP_FLAT, alphas[0]), (1, _nat.STEP_EDGE, alphas[1]), (2, _nat.STEP_FEATURE, alphas[2]))
        self._run_fused(iterations, k, k_update, d, phases, angle)

    def thesisDenoise(self, iterations: int = 2, alphas=DEFAULT_ALPHAS, d: float = None,
                      step_clamp_factor: float = 20000.0, k: int = 2 ** 4, k_update: int = 8, angle: float = None):
        """The thesis-results driver ("Ours", PostProcessing.ipynb:1069-1090): per iteration the feature decomposition,
        then flat_step (alpha[0]) on flat points and feature_step (alphas[1], alphas[2]) on edge and corner points, all
        computed from the iteration's input positions (Jacobi across classes: temp_pos = pos.clone()), with the per-step
        clamp at d * step_clamp_factor (effectively off) and a GLOBAL clamp: a point takes its new position only while
        it stays within d of its position when this call started (mask = ||temp_pos - original_pos|| < d), else it
        keeps its current one.  d defaults to 2 x the mean kNN(6) edge length, as in the notebook."""
        if d is None:
            d = 2 * float(self.meanEdgeLength())
        phases = ((0, _nat.STEP_FLAT, alphas[0]), (1, _nat.STEP_FEATURE, alphas[1]), (2, _nat.STEP_FEATURE, alphas[2]))
        g = self.graph
        GeneralUtils.validateAttributes(g, ["pos", "n"])
        fused = self._fused_for(max(k, k_update))
        fused.load(g.pos, g.n)
        params = _nat.make_params(k=k, k_update=k_update, rho=angle, d=float(d) * step_clamp_factor, phases=phases,
                                  jacobi=True, clamp_global=float(d))
        fused.iterate(params, iterations)
        dev = _nat.device()
        pos_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
        n_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
        fused.store(pos_out, n_out)
        with torch.no_grad():
            g.pos.copy_(pos_out.to(g.pos.dtype))
        g.n = n_out.to(device=g.pos.device, dtype=g.pos.dtype)

    def cpsdDenoise(self, iterations: int = 50, d: float = None, alphas=(0.1, 1.0, 1.0), rho: float = 0.9,
                    tau: float = 0.3, step_clamp_factor: float = 20000.0, k_update: int = 8, fused: bool = True):
        """The CPSD ("Martin") comparison driver of the thesis results (PostProcessing.ipynb:1041-1062): per iteration
        getMartinFeatureDecomposition(r=d) (radius selection of the CURRENT positions against the frozen snapshot,
        normal-filtered NVT, VU smoothing, normal-filtered PVT), VU classes (tau), kNN(k_update), then flat_step /
        edge_step (PVT smallest eigenvector) / corner_step with alphas and the per-step clamp at d * step_clamp_factor,
        all from the iteration's input positions (temp_pos = pos.clone()), and the GLOBAL clamp against the positions at
        the start of the call (mask = ||temp_pos - original_pos|| < d).  graph.pos is updated in place (masked),
        graph.n rebound to f_n.  d defaults to 2 x the mean kNN(6) edge length.
        fused (default): the whole loop in one library call (pcd_cpsd_iterate, every step on the device); False: the
        same operators op by op through the drop-in classes (the cross-check)."""
        g = self.graph
        GeneralUtils.validateAttributes(g, ["pos", "n"])
        if d is None:
            d = 2 * float(self.meanEdgeLength())
        d = float(d)
        if fused:
            dn = self._fused_for(k_update)
            dn.load(g.pos, g.n)
            dn.cpsd_iterate(_nat.make_cpsd_params(r=d, d=d, rho=rho, tau=tau, step_clamp=d * step_clamp_factor,
                                                  alphas=alphas, k_update=k_update), iterations)
            dev = _nat.device()
            pos_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
            n_out = torch.empty((g.num_nodes, 3), dtype=torch.float32, device=dev)
            dn.store(pos_out, n_out)
            with torch.no_grad():
                g.pos.copy_(pos_out.to(g.pos.dtype))          # in place: keeps pointcloud.v aliased
            g.n = n_out.to(device=g.pos.device, dtype=g.pos.dtype)
            return
        original_pos = g.pos.clone()
        den = self.denoiser
        for _ in range(iterations):
            decomposition, f_n = self.getMartinFeatureDecomposition(r=d, rho=rho)
            classes = decomposition.getVUFeatures(tau=tau)
            selection = self.selector.getKNNSelection(k=k_update)
            temp_pos = g.pos.clone()
            for key in range(3):
                indices = (classes == key).nonzero().flatten()
                if indices.size(0) == 0:
                    continue
                sel = selection.filter(indices)
                if key == 0:
                    new_pos = den.flat_step(sel, f_n, d * step_clamp_factor, alphas[key])
                elif key == 1:
                    new_pos = den.edge_step(sel, f_n, decomposition.eigvec[..., 0], d * step_clamp_factor, alphas[key])
                else:
                    new_pos = den.corner_step(sel, f_n, d * step_clamp_factor, alphas[key])
                temp_pos[indices] = new_pos.to(temp_pos.dtype)
            mask = (temp_pos - original_pos).norm(dim=1) < d
            with torch.no_grad():
                g.pos[mask] = temp_pos[mask]
            g.n = f_n

    def denoiseUntilMinimumError(self, gt_pos: torch.Tensor, strategy: dict, k: int = 7,
                                 alpha: list = [0.02, 0.02, 0.1], d: float = 200,
                                 error_funcs: list[Callable] = [TorchUtils.PaperDistance], N: int = 2 ** 4):
        """Processor.py:141-185: iterate while error_funcs[0] decreases; same object flow for the returned tensor."""
        _graph = self.graph
        phases = []
        for key, func in strategy.items():
            name = getattr(func, "__name__", None)
            if name not in STEP_KINDS:
                raise ValueError(f"strategy[{key}] = {func!r} is not a Denoiser step")
            phases.append((int(key), STEP_KINDS[name], float(alpha[key])))
        noisy_graph_pos = _graph.pos.clone()
        noisy_graph_n = _graph.n.clone()
        i = 0
        previous_pos = noisy_graph_pos
        current_pos = previous_pos
        previous_error = [f(gt_pos, _graph.pos) + 200 for f in error_funcs]
        current_error = [f(gt_pos, _graph.pos) for f in error_funcs]
        while current_error[0].mean(dim=0) < previous_error[0].mean(dim=0):
            self._run_fused(1, N, k, d, phases)
            error = [f(gt_pos, _graph.pos) for f in error_funcs]
            previous_error = current_error
            current_error = error
            previous_pos = current_pos
            current_pos = _graph.pos
            i += 1
        _graph.pos = noisy_graph_pos
        _graph.n = noisy_graph_n
        return previous_pos, previous_error, i - 1

    def preprocessPointcloud(self, k: int = 12, noise_level: float = 0.3, generator: torch.Generator = None):
        """Processor.py:187-199: PCA normals, noise along them, PCA normals again + MST orientation."""
        _graph = self.graph
        _gb = self.graphBuilder
        _graph.edge_index = _gb.getKNNEdgeIndex(k)
        _gb.setAndFlipNormals(flip=False)
        l = TorchUtils.averageEdgeLength(_graph.pos, _graph.edge_index)
        self.noise.generateNoise(noise_level, l, keepNormals=False, generator=generator)
        _gb.setAndFlipNormals(flip=True)
