"""TEST INFRASTRUCTURE: a CPU engine for the spatial-slab driver (pcd_slab.SlabDenoiser), built from the oracle.

It mirrors libpcd's staged fused loop (pcd_denoiser_stage, include/pcd.h) on one rank's local snapshot:
active (owned) rows are queried and updated, halo rows are only read and are overwritten by the driver's exchange.
Used by tests/test_slab.py to check the multi-rank orchestration (halo routes, exchange order, global reductions)
with world_size 2 over gloo on the CPU, against the single-process oracle.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pcd_native as nat  # noqa: E402  (constants and the params struct only; no library calls)
from oracle import pcd_oracle as O  # noqa: E402

F32 = np.float32


class CpuSlabEngine:
    def __init__(self, local_pos, local_n, owned_local, k_max, coverage):
        self.snap = local_pos.numpy().astype(F32)
        self.pos = self.snap.copy()
        self.nrm = local_n.numpy().astype(F32).copy()
        self.fn = np.zeros_like(self.nrm)
        self.edge = np.zeros_like(self.nrm)
        self.cls = np.full(len(self.pos), 255, np.int64)
        self.knn = O.FrozenKNN(self.snap)
        self.active = np.sort(owned_local.numpy())
        self.idx = None
        self.lo, self.hi = np.asarray(coverage[0], np.float64), np.asarray(coverage[1], np.float64)
        self.err = 0
        self.red4 = torch.zeros(4, dtype=torch.float64)
        self.red1 = torch.zeros(1, dtype=torch.float32)
        self.centre = {}

    def rows(self, local_idx):
        return local_idx.clone()

    def _class_rows(self, params, ph):
        a = self.active
        return a[self.cls[a] == params.phase_class[ph]]

    def stage(self, params, stage, phase=0, red=None):
        k, ku = params.k, params.k_update
        a = self.active
        if stage == nat.STAGE_KNN_NVT1:
            kstore = max(k, ku)
            idx, dist = self.knn.query(self.pos[a], kstore)
            self.idx = np.zeros((len(self.pos), kstore), np.int64)
            self.idx[a] = idx
            r = dist[:, -1] * (1 + 1e-6)
            q = self.pos[a].astype(np.float64)
            if ((q - r[:, None] < self.lo) | (q + r[:, None] > self.hi)).any():
                self.err |= 2
            w, v = O.better_filtered_nvt(self.pos, self.nrm, a, idx[:, :k], params.rho)
            self.fn[a] = O.vu_smoothed_normals(w, v, self.nrm[a], params.tau, params.damp)
        elif stage == nat.STAGE_NVT2:
            w, v = O.better_filtered_nvt(self.pos, self.fn, a, self.idx[a, :k], params.rho)
            self.cls[a] = O.classes(w, params.class_scale)
            self.edge[a] = v[..., 0]
        elif stage == nat.STAGE_PHASE_SUM:
            rows = self._class_rows(params, phase)
            vj = self.pos[self.idx[rows, :ku]].reshape(-1, 3).astype(np.float64)
            red.copy_(torch.tensor([vj[:, 0].sum(), vj[:, 1].sum(), vj[:, 2].sum(), float(len(vj))]))
        elif stage == nat.STAGE_PHASE_CENTRE:
            s = red.numpy()
            self.centre[phase] = (s[:3] / s[3]).astype(F32)
        elif stage == nat.STAGE_PHASE_MAXDIST:
            rows = self._class_rows(params, phase)
            vj = self.pos[self.idx[rows, :ku]].reshape(-1, 3)
            m = O.norm3(vj - self.centre[phase]).max() if len(vj) else F32(0)
            red.copy_(torch.tensor([float(m)], dtype=torch.float32))
        elif stage == nat.STAGE_PHASE_APPLY:
            rows = self._class_rows(params, phase)
            kind, alpha, d = params.phase_kind[phase], params.phase_alpha[phase], params.d
            new = self.pos.copy()
            if len(rows):
                nbr = self.idx[rows, :ku]
                delta = None if red is None else F32(red.item())
                if kind == nat.STEP_FLAT:
                    out = O.flat_step(self.pos, self.fn, rows, nbr, d, alpha, delta=delta)
                elif kind == nat.STEP_EDGE:
                    out = O.edge_step(self.pos, self.fn, self.edge, rows, nbr, d, alpha)
                elif kind == nat.STEP_FEATURE:
                    out = O.feature_step(self.pos, self.fn, rows, nbr, d, alpha)
                elif kind == nat.STEP_CORNER:
                    out = O.corner_step(self.pos, self.fn, rows, nbr, d, alpha)
                elif kind == nat.STEP_NEW:
                    out = O.new_step(self.pos, self.fn, rows, nbr, d, alpha, delta=delta)
                else:
                    out = self.pos[rows]
                new[rows] = out
            self.pos = new
        elif stage == nat.STAGE_FINISH:
            self.nrm, self.fn = self.fn, self.nrm

    def _field(self, fld):
        return {nat.FIELD_POS: self.pos, nat.FIELD_NRM: self.nrm, nat.FIELD_FN: self.fn}[fld]

    def pack(self, fld, rows):
        f = self._field(fld)[rows.numpy()]
        return torch.from_numpy(np.concatenate([f, np.zeros((len(f), 1), F32)], 1))

    def unpack(self, fld, rows, data):
        self._field(fld)[rows.numpy()] = data[:, :3].numpy()

    def check(self):
        if self.err:
            raise nat.PcdError("halo too thin")

    def status(self):
        return self.err

    def set_state(self, local_idx, pos, n):
        li = local_idx.numpy()
        self.pos[li] = pos.numpy()
        self.nrm[li] = n.numpy()

    def classes(self):
        return torch.from_numpy(self.cls.copy())

    def store(self):
        return torch.from_numpy(self.pos.copy()), torch.from_numpy(self.nrm.copy())


class CpuMeshEngine:
    """Mesh.updateVertices' Jacobi sweep on one rank's local mesh by the oracle (float64), for pcd_slab.MeshSlabs."""

    def __init__(self, v, f, fn):
        self.v = torch.as_tensor(v, dtype=torch.float64).clone()
        self.f = np.asarray(f, np.int64)
        self.fn = np.asarray(fn, np.float64)

    def sweep(self):
        self.v = torch.from_numpy(O.mesh_update(self.v.numpy(), self.f, self.fn, k=1))


class CpuSlabEngineDiag(CpuSlabEngine):
    """The oracle engine with libpcd's coverage diagnostics (pcd_denoiser_coverage_excess, sphere-less rows only):
    a failed check sets bits 2 and 4 and records the farthest reach of a k-ball past the coverage box, so the driver
    grows the band by what it lacked instead of by halo_growth."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.excess = 0.0

    def stage(self, params, stage, phase=0, red=None):
        if stage == nat.STAGE_KNN_NVT1:
            kstore = max(params.k, params.k_update)
            a = self.active
            _, dist = self.knn.query(self.pos[a], kstore)
            r = dist[:, -1] * (1 + 1e-6)
            q = self.pos[a].astype(np.float64)
            ex = np.maximum(self.lo - (q - r[:, None]), (q + r[:, None]) - self.hi).max() if len(a) else 0.0
            if ex > 0:
                self.err |= 2 | 4
                self.excess = max(self.excess, float(ex))
        super().stage(params, stage, phase, red)

    def coverage_excess(self):
        return (self.excess if self.err & 4 else 0.0), 0.0
