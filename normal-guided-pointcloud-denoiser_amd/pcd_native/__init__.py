"""ctypes binding of ``libpcd.so`` -- the C-ABI declared in ``include/pcd.h``.

This is the only module that talks to the native library.  Every compute call of the drop-in classes under
``Pointcloud/Modules`` and ``PatchGeneration/Modules`` goes through here and runs a hand-written HIP kernel on the
current HIP device.  There is NO CPU fallback: if the library or a HIP device is missing, the call raises.
PyTorch is used for device memory, dtype/shape plumbing and the current stream only.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int64, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCD_LIB", os.path.join(os.path.dirname(_HERE), "libpcd.so"))

PCD_OK, PCD_ERR_ARG, PCD_ERR_OOM, PCD_ERR_HIP, PCD_ERR_STATE, PCD_ERR_RCCL = 0, -1, -2, -3, -4, -5
DT_F32, DT_F64, DT_I32 = 0, 1, 2
OP_SUM, OP_MAX = 0, 1
COMM_HOST, COMM_RCCL = 0, 1
FIELD_POS, FIELD_NRM, FIELD_FN, FIELD_EDGE = 0, 1, 2, 3
(STAGE_KNN_NVT1, STAGE_NVT2, STAGE_PHASE_SUM, STAGE_PHASE_CENTRE, STAGE_PHASE_MAXDIST, STAGE_PHASE_APPLY,
 STAGE_FINISH) = range(7)
STEP_FLAT, STEP_EDGE, STEP_FEATURE, STEP_CORNER, STEP_NEW, STEP_DUMMY = range(6)


class PcdError(RuntimeError):
    """A native call failed (HIP error, OOM, bad state)."""


class _GridInfo(ctypes.Structure):
    _fields_ = [("n", c_int64), ("cells", c_int64), ("table_slots", c_int64), ("cell", c_float),
                ("origin", c_float * 3), ("dims", ctypes.c_int32 * 3)]


class CpsdParams(ctypes.Structure):
    """Mirror of ``pcd_cpsd_params`` (include/pcd.h)."""
    _fields_ = [("r", c_float), ("rho", c_float), ("tau", c_float), ("damp", c_float), ("d", c_float),
                ("step_clamp", c_float), ("alpha", c_float * 3), ("k_update", c_int)]


class DenoiseParams(ctypes.Structure):
    """Mirror of ``pcd_denoise_params`` (include/pcd.h)."""
    _fields_ = [("k", c_int), ("k_update", c_int), ("rho", c_float), ("tau", c_float), ("damp", c_float),
                ("class_scale", c_float), ("d", c_float), ("nphases", c_int), ("phase_class", c_int * 3),
                ("phase_kind", c_int * 3), ("phase_alpha", c_float * 3), ("jacobi", c_int), ("clamp_global", c_float)]


# name -> (restype, argtypes); the exact export list of include/pcd.h
_SIGS = {
    "pcd_last_error": (ctypes.c_char_p, []),
    "pcd_version": (c_int, []),
    "pcd_build_id": (ctypes.c_char_p, []),
    "pcd_max_k": (c_int, []),
    "pcd_denoise_params_size": (c_int, []),
    "pcd_grid_build": (c_int, [c_void_p, c_int64, c_int, c_float, c_void_p, c_void_p, POINTER(c_void_p)]),
    "pcd_grid_params": (c_int, [c_void_p, c_int64, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    "pcd_grid_rebuild": (c_int, [c_void_p, c_int, c_float, c_void_p, POINTER(c_void_p)]),
    "pcd_grid_destroy": (c_int, [c_void_p]),
    "pcd_grid_get_info": (c_int, [c_void_p, POINTER(_GridInfo)]),
    "pcd_grid_perm": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_knn": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pcd_knn_stats": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p]),
    "pcd_radius_count": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "pcd_radius_fill": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_nvt_normal_csr": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p,
                                   c_void_p, c_void_p]),
    "pcd_pvt_normal_csr": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_float,
                                   c_void_p, c_void_p, c_void_p]),
    "pcd_nvt_csr": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p,
                            c_void_p, c_void_p]),
    "pcd_vu_smooth": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p, c_void_p]),
    "pcd_classify": (c_int, [c_void_p, c_int64, c_float, c_void_p, c_void_p, c_void_p]),
    "pcd_pca_dense": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "pcd_eigh3_batch": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "pcd_step_csr": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                             c_float, c_float, c_void_p, c_void_p]),
    "pcd_edge_length_sum": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_nn_dist": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "pcd_mesh_update": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_void_p]),
    "pcd_mesh_update_f32": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int,
                                    c_void_p]),
    "pcd_mesh_vta": (c_int, [c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p, c_int, c_void_p]),
    "pcd_denoiser_create": (c_int, [c_void_p, c_int, POINTER(c_void_p)]),
    "pcd_denoiser_destroy": (c_int, [c_void_p]),
    "pcd_denoiser_load": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_iterate": (c_int, [c_void_p, POINTER(DenoiseParams), c_int, c_void_p]),
    "pcd_denoiser_store": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_set_timing": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_reset_seed": (c_int, [c_void_p]),
    "pcd_denoiser_set_seeding": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_set_anchoring": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_set_windows": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_anchor_stats": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_tile_stats": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_check": (c_int, [c_void_p, c_void_p]),
    "pcd_denoiser_status": (c_int, [c_void_p, POINTER(c_int), c_void_p]),
    "pcd_denoiser_coverage_excess": (c_int, [c_void_p, POINTER(c_float), POINTER(c_float), c_void_p]),
    "pcd_denoiser_lists": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "pcd_denoiser_set_probe": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_probe_store": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_set_rows": (c_int, [c_void_p, c_void_p, c_int64]),
    "pcd_denoiser_set_coverage": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_set_coverage_spheres": (c_int, [c_void_p, c_void_p, c_void_p]),
    "pcd_denoiser_stage": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "pcd_denoiser_pack": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_denoiser_unpack": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_denoiser_get_timing": (c_int, [c_void_p, POINTER(c_float), c_int, POINTER(c_int)]),
    "pcd_cpsd_iterate": (c_int, [c_void_p, POINTER(CpsdParams), c_int, c_void_p]),
    "pcd_comm_id_bytes": (c_int, []),
    "pcd_comm_id": (c_int, [c_void_p]),
    "pcd_comm_create": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p)]),
    "pcd_comm_create_host": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p)]),
    "pcd_comm_destroy": (c_int, [c_void_p]),
    "pcd_comm_info": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "pcd_comm_sendrecv": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int, c_void_p, c_int64, c_void_p]),
    "pcd_allreduce_scalars": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "pcd_denoiser_set_routes": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p]),
    "pcd_halo_exchange": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "pcd_denoiser_set_readset": (c_int, [c_void_p, c_int]),
    "pcd_denoiser_readset_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "pcd_slab_iterate": (c_int, [c_void_p, c_void_p, POINTER(DenoiseParams), c_int, c_void_p]),
    "pcd_orient_normals_mst": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64]),
    "pcd_orient_normals_mst_gpu": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p]),
    "pcd_host_eigh3": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_host_vu_smooth": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p]),
    "pcd_host_solve3": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_host_inv3": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "pcd_host_step_csr": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float,
                                  c_float, c_float, c_void_p]),
    "pcd_host_nvt_tensor": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p]),
}

_lib = None


def lib():
    """Load libpcd.so once (raises ImportError with the build hint if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"pcd: native library not found at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "or `make -C normal-guided-pointcloud-denoiser_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name, None)
            if f is None:
                if "PCD_LIB" in os.environ:     # an older experiment build (A/B): its missing entry points stay unbound
                    continue
                raise ImportError(f"pcd: {LIB_PATH} does not export {name}: rebuild it")
            f.restype = res
            f.argtypes = args
        # the params mirror must match the library's struct (a shorter one would be read past its end)
        if ctypes.sizeof(DenoiseParams) != L.pcd_denoise_params_size():
            raise ImportError(f"pcd: DenoiseParams mirror is {ctypes.sizeof(DenoiseParams)} B, the library's "
                              f"pcd_denoise_params is {L.pcd_denoise_params_size()} B -- rebuild or update the mirror")
        _lib = L
    return _lib


def build_id() -> str:
    """The loaded library's build id (pcd_build_id: a hash of its sources and extra flags)."""
    return lib().pcd_build_id().decode()


def exported_symbols():
    return list(_SIGS.keys())


def check(status: int, what: str = ""):
    if status == PCD_OK:
        return
    msg = lib().pcd_last_error().decode(errors="replace")
    if status == PCD_ERR_ARG:
        raise ValueError(f"pcd: {what}: {msg}")
    raise PcdError(f"pcd: {what} failed ({status}): {msg}")


# ----------------------------------------------------------------------------------------------- device plumbing
def device() -> torch.device:
    """The HIP device every kernel runs on.  Raises if there is none (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("pcd: no HIP (ROCm) device available -- the denoiser runs its kernels on MI355X only")
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None):
    return None if t is None else c_void_p(t.data_ptr())


def on_device(t: torch.Tensor, dtype=None) -> torch.Tensor:
    """Contiguous copy/view of `t` on the HIP device with the requested dtype."""
    dev = device()
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if t.device != dev:
        t = t.to(dev, non_blocking=False)
    return t.contiguous()


def f32(t):
    return on_device(t, torch.float32)


def i64(t):
    return on_device(t, torch.int64)


# ----------------------------------------------------------------------------------------------- objects
class Grid:
    """Frozen snapshot + kNN index (pcd_grid).  Mirrors the KDTree made in Selector.__init__."""

    def __init__(self, xyz: torch.Tensor, k_hint: int = 16, cell: float = 0.0, origin=None):
        """origin: optional (3,) lattice origin (needs cell > 0), see pcd_grid_build."""
        L = lib()
        x = f32(xyz)
        assert x.dim() == 2 and x.size(1) == 3
        self._keep = x
        h = c_void_p()
        org = None
        if origin is not None:
            org = (ctypes.c_float * 3)(*[float(v) for v in origin])
        check(L.pcd_grid_build(ptr(x), x.size(0), int(k_hint), float(cell), org, c_void_p(stream_ptr()),
                               ctypes.byref(h)), "pcd_grid_build")
        self.handle = h
        self.n = x.size(0)
        self.k_hint = int(k_hint) if cell <= 0 else 0
        self._keep = None

    def rebuild(self, k_hint: int) -> "Grid":
        """A grid over this grid's own frozen snapshot with cells of ~k_hint/2 points (pcd_grid_rebuild)."""
        h = c_void_p()
        check(lib().pcd_grid_rebuild(self.handle, int(k_hint), 0.0, c_void_p(stream_ptr()), ctypes.byref(h)),
              "pcd_grid_rebuild")
        g = Grid.__new__(Grid)
        g.handle, g.n, g.k_hint, g._keep = h, self.n, int(k_hint), None
        return g

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib is not None:
            _lib.pcd_grid_destroy(h)
            self.handle = None

    def info(self) -> dict:
        gi = _GridInfo()
        check(lib().pcd_grid_get_info(self.handle, ctypes.byref(gi)), "pcd_grid_get_info")
        return {"n": gi.n, "cells": gi.cells, "table_slots": gi.table_slots, "cell": gi.cell,
                "origin": list(gi.origin), "dims": list(gi.dims)}

    def perm(self) -> torch.Tensor:
        out = torch.empty(self.n, dtype=torch.int32, device=device())
        check(lib().pcd_grid_perm(self.handle, ptr(out), c_void_p(stream_ptr())), "pcd_grid_perm")
        return out

    def knn(self, q: torch.Tensor, k: int, exclude_self: bool = False, with_d2: bool = False, idx_bits: int = 64,
            sorted_ids: bool = False):
        q = f32(q)
        nq = q.size(0)
        idx = torch.empty((nq, k), dtype=torch.int64 if idx_bits == 64 else torch.int32, device=q.device)
        d2 = torch.empty((nq, k), dtype=torch.float32, device=q.device) if with_d2 else None
        check(lib().pcd_knn(self.handle, ptr(q), nq, int(k), ptr(idx), idx_bits, int(sorted_ids), int(exclude_self),
                            ptr(d2), c_void_p(stream_ptr())), "pcd_knn")
        return (idx, d2) if with_d2 else idx

    def knn_stats(self, q: torch.Tensor, k: int, batched: bool = False) -> dict:
        """Per-query averages of the kNN search work (diagnostic build of the search; batched or insertion)."""
        q = f32(q)
        out = torch.zeros(6, dtype=torch.int64, device=q.device)
        check(lib().pcd_knn_stats(self.handle, ptr(q), q.size(0), int(k), int(bool(batched)), ptr(out),
                                  c_void_p(stream_ptr())),
              "pcd_knn_stats")
        v = out.cpu().double() / max(q.size(0), 1)
        names = ["cells_considered", "cells_probed", "cells_found", "candidates", "inserts", "extra_rings"]
        return {nm: round(float(x), 2) for nm, x in zip(names, v)}

    def radius_counts(self, q: torch.Tensor, radii: torch.Tensor) -> torch.Tensor:
        """Member counts of the balls of radii[i] around q[i] (pcd_radius_count), int64 [nq]."""
        q = f32(q)
        r = f32(radii)
        counts = torch.empty(q.size(0), dtype=torch.int64, device=q.device)
        check(lib().pcd_radius_count(self.handle, ptr(q), q.size(0), ptr(r), ptr(counts), c_void_p(stream_ptr())),
              "pcd_radius_count")
        return counts

    def radius(self, q: torch.Tensor, radii: torch.Tensor):
        """Members of the ball of radii[i] around q[i] (original snapshot ids, ascending): (slices int64 [nq+1],
        j int64 [total]) -- scipy query_ball_point semantics (pcd_radius_count / pcd_radius_fill)."""
        q = f32(q)
        r = f32(radii)
        nq = q.size(0)
        counts = torch.empty(nq, dtype=torch.int64, device=q.device)
        check(lib().pcd_radius_count(self.handle, ptr(q), nq, ptr(r), ptr(counts), c_void_p(stream_ptr())),
              "pcd_radius_count")
        slices = torch.zeros(nq + 1, dtype=torch.int64, device=q.device)
        torch.cumsum(counts, 0, out=slices[1:])
        total = int(slices[-1])
        j = torch.empty(total, dtype=torch.int64, device=q.device)
        check(lib().pcd_radius_fill(self.handle, ptr(q), nq, ptr(r), ptr(slices), total, ptr(j),
                                    c_void_p(stream_ptr())), "pcd_radius_fill")
        return slices, j

    def nn(self, q: torch.Tensor):
        q = f32(q)
        d2 = torch.empty(q.size(0), dtype=torch.float32, device=q.device)
        idx = torch.empty(q.size(0), dtype=torch.int64, device=q.device)
        check(lib().pcd_nn_dist(self.handle, ptr(q), q.size(0), ptr(d2), ptr(idx), c_void_p(stream_ptr())),
              "pcd_nn_dist")
        return d2, idx


class FusedDenoiser:
    """Persistent buffers of the fused loop (pcd_denoiser) bound to one Grid."""

    def __init__(self, grid: Grid, k_max: int):
        self.grid = grid
        h = c_void_p()
        check(lib().pcd_denoiser_create(grid.handle, int(k_max), ctypes.byref(h)), "pcd_denoiser_create")
        self.handle = h
        self.k_max = k_max

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib is not None:
            _lib.pcd_denoiser_destroy(h)
            self.handle = None

    def load(self, pos: torch.Tensor, n: torch.Tensor):
        pos, n = f32(pos), f32(n)
        check(lib().pcd_denoiser_load(self.handle, ptr(pos), ptr(n), c_void_p(stream_ptr())), "pcd_denoiser_load")

    def iterate(self, params: DenoiseParams, iterations: int):
        check(lib().pcd_denoiser_iterate(self.handle, ctypes.byref(params), int(iterations), c_void_p(stream_ptr())),
              "pcd_denoiser_iterate")

    def store(self, pos=None, n=None, classes=None, edge_vectors=None):
        check(lib().pcd_denoiser_store(self.handle, ptr(pos), ptr(n), ptr(classes), ptr(edge_vectors),
                                       c_void_p(stream_ptr())), "pcd_denoiser_store")

    def lists(self, cols: int) -> torch.Tensor:
        """The kNN lists of the last iteration (original indices, caller order): int64 [N, cols]."""
        out = torch.empty((self.grid.n, int(cols)), dtype=torch.int64, device=device())
        check(lib().pcd_denoiser_lists(self.handle, ptr(out), int(cols), c_void_p(stream_ptr())), "pcd_denoiser_lists")
        return out

    def set_probe(self, enable=True):
        """NVT2 parity probe on / off (pcd_denoiser_set_probe)."""
        check(lib().pcd_denoiser_set_probe(self.handle, int(bool(enable))), "pcd_denoiser_set_probe")

    def probe(self) -> torch.Tensor:
        """(λ0, λ1, λ2, Σw) of the last NVT2 stage per point, caller order: float32 [N, 4]."""
        out = torch.empty((self.grid.n, 4), dtype=torch.float32, device=device())
        check(lib().pcd_denoiser_probe_store(self.handle, ptr(out), c_void_p(stream_ptr())), "pcd_denoiser_probe_store")
        return out

    def set_seeding(self, enable=True):
        check(lib().pcd_denoiser_set_seeding(self.handle, int(bool(enable))), "pcd_denoiser_set_seeding")

    def set_anchoring(self, enable=True):
        check(lib().pcd_denoiser_set_anchoring(self.handle, int(bool(enable))), "pcd_denoiser_set_anchoring")

    def set_windows(self, enable=True):
        check(lib().pcd_denoiser_set_windows(self.handle, int(bool(enable))), "pcd_denoiser_set_windows")

    def redo_rows(self) -> int:
        """Rows re-anchored by the last anchored kNN stage (-1: none ran)."""
        v = ctypes.c_int64(0)
        check(lib().pcd_denoiser_anchor_stats(self.handle, ctypes.byref(v), c_void_p(stream_ptr())),
              "pcd_denoiser_anchor_stats")
        return v.value

    def tile_stats(self) -> dict:
        """Counters of the last anchored kNN stage (pcd_denoiser_tile_stats)."""
        v = (ctypes.c_int64 * 4)()
        check(lib().pcd_denoiser_tile_stats(self.handle, v, c_void_p(stream_ptr())), "pcd_denoiser_tile_stats")
        return {"rows": v[0], "spilled": v[1], "spilled_big_box": v[2], "spilled_ambiguous": v[3]}

    def reset_seed(self):
        check(lib().pcd_denoiser_reset_seed(self.handle), "pcd_denoiser_reset_seed")

    def set_timing(self, on):
        """False / True: off / every stage (TIMING_SLOTS); 2: the K1 stage only (one slot, K1's ms)."""
        check(lib().pcd_denoiser_set_timing(self.handle, int(on)), "pcd_denoiser_set_timing")

    def check(self):
        check(lib().pcd_denoiser_check(self.handle, c_void_p(stream_ptr())), "pcd_denoiser_check")

    def status(self) -> int:
        """Device error word (bit 0: invalid list entry, bit 1: a k-ball left the coverage box -- bit 2: a sphere-less
        row, bit 3: a coverage-sphere row), not raising."""
        v = c_int(0)
        check(lib().pcd_denoiser_status(self.handle, ctypes.byref(v), c_void_p(stream_ptr())), "pcd_denoiser_status")
        return v.value

    def coverage_excess(self) -> tuple:
        """(band_excess, sphere_ratio) of the failed coverage checks (pcd_denoiser_coverage_excess): how far the
        farthest sphere-less k-ball reached past the coverage box, the largest (|q - c| + d_k) / R of a sphere row
        (0: no such failure)."""
        b, s = c_float(0.0), c_float(0.0)
        check(lib().pcd_denoiser_coverage_excess(self.handle, ctypes.byref(b), ctypes.byref(s), c_void_p(stream_ptr())),
              "pcd_denoiser_coverage_excess")
        return float(b.value), float(s.value)

    # ---- spatial slabs: active rows, coverage, staged iteration, halo pack/unpack (include/pcd.h)
    @staticmethod
    def _rows_i32(rows: torch.Tensor) -> torch.Tensor:
        """Row lists go to the C-ABI as int32_t*: any integer tensor is converted on the HIP device (the converted
        tensor must be kept alive by the caller until the launch has consumed it)."""
        assert not rows.is_floating_point() and not rows.is_complex(), "row indices must be an integer tensor"
        return on_device(rows.reshape(-1), torch.int32)

    def set_rows(self, rows):
        """rows: integer tensor of spatial-order rows (converted to int32 on the device and kept alive here), or
        None for all rows."""
        self._rows = None if rows is None else self._rows_i32(rows)
        n = 0 if rows is None else self._rows.numel()
        check(lib().pcd_denoiser_set_rows(self.handle, ptr(self._rows), n), "pcd_denoiser_set_rows")

    def set_coverage(self, lo=None, hi=None):
        if lo is None:
            check(lib().pcd_denoiser_set_coverage(self.handle, None, None), "pcd_denoiser_set_coverage")
            return
        lo3 = (c_float * 3)(*[float(v) for v in lo])
        hi3 = (c_float * 3)(*[float(v) for v in hi])
        check(lib().pcd_denoiser_set_coverage(self.handle, lo3, hi3), "pcd_denoiser_set_coverage")

    def set_coverage_spheres(self, radii=None):
        """Per-point coverage spheres (float32 [n], caller order, 0 = none; None clears): pcd_denoiser_set_coverage_spheres."""
        r = None if radii is None else f32(radii)
        if r is not None:
            assert r.dim() == 1 and r.numel() == self.grid.n
        check(lib().pcd_denoiser_set_coverage_spheres(self.handle, ptr(r), c_void_p(stream_ptr())),
              "pcd_denoiser_set_coverage_spheres")
        if r is not None:
            torch.cuda.current_stream().synchronize()

    def stage(self, params: DenoiseParams, stage: int, phase: int = 0, red: torch.Tensor = None):
        check(lib().pcd_denoiser_stage(self.handle, ctypes.byref(params), int(stage), int(phase), ptr(red),
                                       c_void_p(stream_ptr())), "pcd_denoiser_stage")

    def pack(self, field: int, rows: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        rows = self._rows_i32(rows)
        n = rows.numel()
        if out is None:
            out = torch.empty((n, 4), dtype=torch.float32, device=rows.device)
        assert out.dtype == torch.float32 and out.is_contiguous() and out.shape == (n, 4) and out.device == rows.device
        check(lib().pcd_denoiser_pack(self.handle, int(field), ptr(rows), n, ptr(out), c_void_p(stream_ptr())),
              "pcd_denoiser_pack")
        return out

    def unpack(self, field: int, rows: torch.Tensor, data: torch.Tensor):
        rows = self._rows_i32(rows)
        data = data.contiguous()
        assert data.dtype == torch.float32 and data.shape == (rows.numel(), 4) and data.device == rows.device
        check(lib().pcd_denoiser_unpack(self.handle, int(field), ptr(rows), rows.numel(), ptr(data),
                                        c_void_p(stream_ptr())), "pcd_denoiser_unpack")

    # ---- spatial slabs in one call per iteration (pcd_denoiser_set_routes / pcd_slab_iterate, include/pcd.h)
    def set_routes(self, peers, send_rows, recv_rows, own_lo=None, own_hi=None):
        """peers: list of peer ranks; send_rows / recv_rows: per peer an integer tensor of spatial-order rows.  The
        library copies them.  own_lo / own_hi: the owned slab's box (enables the exchange / compute overlap)."""
        npeers = len(peers)
        pa = (c_int * max(npeers, 1))(*[int(q) for q in peers])
        ns = (c_int64 * max(npeers, 1))(*[int(r.numel()) for r in send_rows])
        nr = (c_int64 * max(npeers, 1))(*[int(r.numel()) for r in recv_rows])
        dev = device()
        cat = lambda rs: (torch.cat([self._rows_i32(r) for r in rs]) if rs and sum(r.numel() for r in rs)
                          else torch.zeros(1, dtype=torch.int32, device=dev))
        sr, rr = cat(send_rows), cat(recv_rows)
        lo3 = None if own_lo is None else (c_float * 3)(*[float(v) for v in own_lo])
        hi3 = None if own_hi is None else (c_float * 3)(*[float(v) for v in own_hi])
        check(lib().pcd_denoiser_set_routes(self.handle, npeers, pa, ns, ptr(sr), nr, ptr(rr), lo3, hi3,
                                            c_void_p(stream_ptr())), "pcd_denoiser_set_routes")

    def cpsd_iterate(self, params: "CpsdParams", iterations: int):
        """The CPSD driver's iterations on the loaded state (pcd_cpsd_iterate)."""
        check(lib().pcd_cpsd_iterate(self.handle, ctypes.byref(params), int(iterations), c_void_p(stream_ptr())),
              "pcd_cpsd_iterate")

    def slab_iterate(self, comm: "Comm", params: DenoiseParams, iterations: int = 1):
        check(lib().pcd_slab_iterate(self.handle, comm.handle, ctypes.byref(params), int(iterations),
                                     c_void_p(stream_ptr())), "pcd_slab_iterate")

    def halo_exchange(self, comm: "Comm", field: int):
        check(lib().pcd_halo_exchange(self.handle, comm.handle, int(field), c_void_p(stream_ptr())),
              "pcd_halo_exchange")

    def set_readset(self, on: bool):
        """slab_iterate moves only the halo rows the lists read (pcd_denoiser_set_readset; default on)."""
        check(lib().pcd_denoiser_set_readset(self.handle, int(bool(on))), "pcd_denoiser_set_readset")

    def readset_stats(self) -> tuple:
        """(iterations, send rows, receive rows) of the read-set exchange since set_routes, summed."""
        it, s, r = c_int64(0), c_int64(0), c_int64(0)
        check(lib().pcd_denoiser_readset_stats(self.handle, ctypes.byref(it), ctypes.byref(s), ctypes.byref(r)),
              "pcd_denoiser_readset_stats")
        return it.value, s.value, r.value

    TIMING_SLOTS = ("anchor_test", "requery", "spill_search", "nvt1", "nvt2", "flat_phase", "edge_phase",
                    "corner_phase", "finish")

    def timing(self):
        """Per-stage ms averaged over the iterations timed since set_timing / the last call (TIMING_SLOTS order)."""
        buf = (c_float * 16)()
        nw = c_int(0)
        check(lib().pcd_denoiser_get_timing(self.handle, buf, 16, ctypes.byref(nw)), "pcd_denoiser_get_timing")
        return [buf[i] for i in range(nw.value)]


# ----------------------------------------------------------------------------------------------- slab transport
_EXCHANGE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, POINTER(c_int), POINTER(c_float), POINTER(c_int64),
                                POINTER(c_float), POINTER(c_int64))
_ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_int, c_int, c_int)


class _HostTransport(ctypes.Structure):
    _fields_ = [("user", c_void_p), ("exchange", _EXCHANGE_FN), ("allreduce", _ALLREDUCE_FN)]


class Comm:
    """The slab transport of libpcd (pcd_comm): RCCL, or host callbacks over a torch.distributed CPU group (gloo)."""

    def __init__(self, handle, keep=None):
        self.handle = handle
        self._keep = keep

    @staticmethod
    def rccl(world: int, rank: int, broadcast) -> "Comm":
        """Collective: rank 0 makes an RCCL unique id, `broadcast(uint8 tensor)` (in place, from rank 0) hands it to
        every rank, and every rank joins the communicator on its current HIP device."""
        L = lib()
        nb = L.pcd_comm_id_bytes()
        buf = (ctypes.c_ubyte * nb)()
        if rank == 0:
            check(L.pcd_comm_id(buf), "pcd_comm_id")
        t = torch.tensor(bytearray(buf), dtype=torch.uint8)
        t = broadcast(t)
        ctypes.memmove(buf, bytes(t.cpu().numpy().tobytes()), nb)
        h = c_void_p()
        check(L.pcd_comm_create(buf, int(world), int(rank), ctypes.byref(h)), "pcd_comm_create")
        return Comm(h)

    @staticmethod
    def host(world: int, rank: int, exchange, allreduce) -> "Comm":
        """exchange(peers, send [ns, 4] f32 array, send_off, recv [nr, 4] array to fill, recv_off) and
        allreduce(buf array, op) over numpy views of the library's host staging buffers (no copies)."""
        import numpy as np

        def _ex(user, npeers, peers, send, soff, recv, roff):
            try:
                P = [peers[q] for q in range(npeers)]
                so = [soff[q] for q in range(npeers + 1)]
                ro = [roff[q] for q in range(npeers + 1)]
                sa = np.ctypeslib.as_array(send, shape=(max(so[-1], 1) * 4,)).reshape(-1, 4)
                ra = np.ctypeslib.as_array(recv, shape=(max(ro[-1], 1) * 4,)).reshape(-1, 4)
                exchange(P, sa, so, ra, ro)
                return 0
            except Exception as e:                              # noqa: BLE001  (reported as a status code)
                import traceback
                traceback.print_exc()
                return 1

        def _ar(user, buf, count, dtype, op):
            try:
                dt = {DT_F32: np.float32, DT_F64: np.float64, DT_I32: np.int32}[dtype]
                arr = np.frombuffer((ctypes.c_char * (count * np.dtype(dt).itemsize)).from_address(buf), dtype=dt)
                allreduce(arr, op)
                return 0
            except Exception:                                   # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1

        cbs = _HostTransport(None, _EXCHANGE_FN(_ex), _ALLREDUCE_FN(_ar))
        h = c_void_p()
        check(lib().pcd_comm_create_host(ctypes.byref(cbs), int(world), int(rank), ctypes.byref(h)),
              "pcd_comm_create_host")
        return Comm(h, keep=(cbs, _ex, _ar))

    def info(self) -> dict:
        """world / rank / transport ("rccl" or "host") as the library's communicator sees them (pcd_comm_info)."""
        w, r, tr = c_int(0), c_int(0), c_int(0)
        check(lib().pcd_comm_info(self.handle, ctypes.byref(w), ctypes.byref(r), ctypes.byref(tr)), "pcd_comm_info")
        return {"world": w.value, "rank": r.value, "transport": "rccl" if tr.value == COMM_RCCL else "host"}

    def sendrecv(self, send_peer: int = -1, send: torch.Tensor = None, recv_peer: int = -1,
                 recv: torch.Tensor = None):
        """Point-to-point copy of contiguous device tensors (pcd_comm_sendrecv): `send` to rank send_peer, `recv`
        filled from rank recv_peer, in place; either side may be absent (peer -1)."""
        for t in (send, recv):
            assert t is None or (t.is_cuda and t.is_contiguous() and (t.numel() * t.element_size()) % 4 == 0)
        sb = 0 if send is None else send.numel() * send.element_size()
        rb = 0 if recv is None else recv.numel() * recv.element_size()
        check(lib().pcd_comm_sendrecv(self.handle, int(send_peer if send is not None else -1), ptr(send), sb,
                                      int(recv_peer if recv is not None else -1), ptr(recv), rb,
                                      c_void_p(stream_ptr())), "pcd_comm_sendrecv")
        return recv

    def allreduce_(self, t: torch.Tensor, op: int = OP_SUM) -> torch.Tensor:
        """In-place all-reduce of a small device tensor (float32 / float64 / int32)."""
        dt = {torch.float32: DT_F32, torch.float64: DT_F64, torch.int32: DT_I32}[t.dtype]
        assert t.is_contiguous() and t.is_cuda
        check(lib().pcd_allreduce_scalars(self.handle, ptr(t), t.numel(), dt, int(op), c_void_p(stream_ptr())),
              "pcd_allreduce_scalars")
        return t

    def destroy(self):
        """pcd_comm_destroy now (every rank at the same point of its program: the RCCL communicator's teardown)."""
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib is not None:
            _lib.pcd_comm_destroy(h)
        self.handle = None

    def __del__(self):
        self.destroy()


def make_cpsd_params(r, d, rho=0.9, tau=0.3, damp=3.0, step_clamp=None, alphas=(0.1, 1.0, 1.0), k_update=8):
    p = CpsdParams()
    p.r, p.rho, p.tau, p.damp, p.d = float(r), float(rho), float(tau), float(damp), float(d)
    p.step_clamp = float(d * 20000.0 if step_clamp is None else step_clamp)
    for a in range(3):
        p.alpha[a] = float(alphas[a])
    p.k_update = int(k_update)
    return p


def make_params(k=16, k_update=8, rho=None, tau=0.3, damp=3.0, class_scale=0.2, d=1.0,
                phases=((0, STEP_FLAT, 1.0), (1, STEP_EDGE, 0.2), (2, STEP_FEATURE, 1.0)), jacobi=False,
                clamp_global=0.0) -> DenoiseParams:
    import math
    p = DenoiseParams()
    p.k, p.k_update = int(k), int(k_update)
    p.rho = float(math.pi * 5 / 12 if rho is None else rho)
    p.tau, p.damp, p.class_scale, p.d = float(tau), float(damp), float(class_scale), float(d)
    p.nphases = len(phases)
    for t, (c, kind, a) in enumerate(phases):
        p.phase_class[t], p.phase_kind[t], p.phase_alpha[t] = int(c), int(kind), float(a)
    p.jacobi = int(bool(jacobi))
    p.clamp_global = float(clamp_global)
    return p


# ----------------------------------------------------------------------------------------------- op wrappers
def nvt_csr(pos, n, ci, off, nbr, rho):
    m = ci.size(0)
    ev = torch.empty((m, 3), dtype=torch.float32, device=pos.device)
    evec = torch.empty((m, 3, 3), dtype=torch.float32, device=pos.device)
    check(lib().pcd_nvt_csr(ptr(pos), ptr(n), pos.size(0), ptr(ci), ptr(off), ptr(nbr), m, float(rho), ptr(ev),
                            ptr(evec), c_void_p(stream_ptr())), "pcd_nvt_csr")
    return ev, evec


def nvt_normal_csr(n, ci, off, nbr, rho):
    m = ci.size(0)
    ev = torch.empty((m, 3), dtype=torch.float32, device=n.device)
    evec = torch.empty((m, 3, 3), dtype=torch.float32, device=n.device)
    check(lib().pcd_nvt_normal_csr(ptr(n), n.size(0), ptr(ci), ptr(off), ptr(nbr), m, float(rho), ptr(ev),
                                   ptr(evec), c_void_p(stream_ptr())), "pcd_nvt_normal_csr")
    return ev, evec


def pvt_normal_csr(pos, n, ci, off, nbr, rho):
    m = ci.size(0)
    ev = torch.empty((m, 3), dtype=torch.float32, device=pos.device)
    evec = torch.empty((m, 3, 3), dtype=torch.float32, device=pos.device)
    check(lib().pcd_pvt_normal_csr(ptr(pos), ptr(n), pos.size(0), ptr(ci), ptr(off), ptr(nbr), m, float(rho),
                                   ptr(ev), ptr(evec), c_void_p(stream_ptr())), "pcd_pvt_normal_csr")
    return ev, evec


def vu_smooth(eigval, eigvec, n, tau, damp):
    out = torch.empty_like(n)
    check(lib().pcd_vu_smooth(ptr(eigval), ptr(eigvec), ptr(n), n.size(0), float(tau), float(damp), ptr(out),
                              c_void_p(stream_ptr())), "pcd_vu_smooth")
    return out


def classify(eigval, scale, want_features=False):
    m = eigval.size(0)
    cls = torch.empty(m, dtype=torch.int64, device=eigval.device)
    feat = torch.empty((m, 3), dtype=torch.float32, device=eigval.device) if want_features else None
    check(lib().pcd_classify(ptr(eigval), m, float(scale), ptr(feat), ptr(cls), c_void_p(stream_ptr())),
          "pcd_classify")
    return cls, feat


def pca_dense(pos, nbr, k):
    n = pos.size(0)
    ev = torch.empty((n, 3), dtype=torch.float32, device=pos.device)
    evec = torch.empty((n, 3, 3), dtype=torch.float32, device=pos.device)
    check(lib().pcd_pca_dense(ptr(pos), n, ptr(nbr), int(k), ptr(ev), ptr(evec), c_void_p(stream_ptr())),
          "pcd_pca_dense")
    return ev, evec


def eigh3_batch(t6, solver=0):
    """Device eigen-solvers of the kernels on t6 (m, 6): solver 0 (LAPACK restatement) -> (w (m,3), V (m,3,3));
    solver 1 (NVT2's Jacobi) -> (w (m,3), y (m,3))."""
    t = f32(t6)
    assert t.dim() == 2 and t.size(1) == 6
    m = t.size(0)
    w = torch.empty((m, 3), dtype=torch.float32, device=t.device)
    vec = torch.empty((m, 3, 3) if solver == 0 else (m, 3), dtype=torch.float32, device=t.device)
    check(lib().pcd_eigh3_batch(ptr(t), m, int(solver), ptr(w), ptr(vec), c_void_p(stream_ptr())), "pcd_eigh3_batch")
    return w, vec


def step_csr(kind, pos, n, edge_vectors, ci, off, nbr, d, alpha):
    m = ci.size(0)
    out = torch.empty((m, 3), dtype=torch.float32, device=pos.device)
    check(lib().pcd_step_csr(int(kind), ptr(pos), ptr(n), ptr(edge_vectors), pos.size(0), ptr(ci), ptr(off),
                             ptr(nbr), m, float(d), float(alpha), ptr(out), c_void_p(stream_ptr())), "pcd_step_csr")
    return out


def edge_length_sum(pos, a, b):
    s = torch.empty(1, dtype=torch.float64, device=pos.device)
    check(lib().pcd_edge_length_sum(ptr(pos), ptr(a), ptr(b), a.size(0), ptr(s), c_void_p(stream_ptr())),
          "pcd_edge_length_sum")
    return s


def mesh_update(v, f, fn, vf, ni, k):
    check(lib().pcd_mesh_update(ptr(v), v.size(0), ptr(f), ptr(fn), f.size(0), ptr(vf), ptr(ni), int(k),
                                c_void_p(stream_ptr())), "pcd_mesh_update")


def mesh_update_f32(v, f, fn, vf, ni, k):
    """fp32 sweeps: v float32 [nv,3] (in place), f int32 [nf,3], fn float32 [nf,3], vf / ni int32 (device)."""
    assert v.dtype == torch.float32 and fn.dtype == torch.float32
    assert f.dtype == torch.int32 and vf.dtype == torch.int32 and ni.dtype == torch.int32
    check(lib().pcd_mesh_update_f32(ptr(v), v.size(0), ptr(f), ptr(fn), f.size(0), ptr(vf), ptr(ni), int(k),
                                    c_void_p(stream_ptr())), "pcd_mesh_update_f32")


def mesh_vta(f: torch.Tensor, nv: int, out_dtype=torch.int64):
    """igl.vertex_triangle_adjacency on the device: (vf [3 nf], ni [nv + 1]) in out_dtype (int32 / int64)."""
    f = on_device(f)
    assert f.dtype in (torch.int32, torch.int64) and f.dim() == 2 and f.size(1) == 3
    nf = f.size(0)
    vf = torch.empty(3 * nf, dtype=out_dtype, device=f.device)
    ni = torch.empty(nv + 1, dtype=out_dtype, device=f.device)
    check(lib().pcd_mesh_vta(ptr(f), 32 if f.dtype == torch.int32 else 64, nf, int(nv), ptr(vf), ptr(ni),
                             32 if out_dtype == torch.int32 else 64, c_void_p(stream_ptr())), "pcd_mesh_vta")
    return vf, ni


def list_cap(k: int) -> int:
    """Columns of the fused loop's stored lists for k = max(k, k_update) (denoise.hip list_cap)."""
    return 8 if k <= 8 else 16 if k <= 16 else 32 if k <= 32 else 64


def fused_k_hint(k_max: int) -> int:
    """Cell size of the fused loop's snapshot index: about one list cap of points per occupied cell (k_hint = 2 x
    the cap) for the anchored searches (cap <= 32).  Measured at 10M points, k = 32 (cap 32), iterations 6-25: 8 points
    a cell 8.16 ms per iteration, 16 a cell 5.77 ms, 32 a cell 5.44 ms, 48 a cell 5.46 ms, 64 a cell 5.57 ms."""
    cap = list_cap(k_max)
    return 2 * cap if cap <= 32 else 0


def grid_params(xyz: torch.Tensor, k_hint: int = 16, cell: float = 0.0):
    """(origin (3,), cell edge) of the lattice pcd_grid_build would use for xyz."""
    x = f32(xyz)
    org = (ctypes.c_float * 3)()
    h = ctypes.c_float()
    check(lib().pcd_grid_params(ptr(x), x.size(0), int(k_hint), float(cell), org, ctypes.byref(h),
                                c_void_p(stream_ptr())), "pcd_grid_params")
    return [org[0], org[1], org[2]], h.value


def host_eigh3(t6):
    """CPU build of the kernels' eigen-decomposition: t6 (m, 6) float32 -> (w (m,3), v (m,3,3))."""
    import numpy as np
    t6 = np.ascontiguousarray(t6, dtype=np.float32)
    m = t6.shape[0]
    w = np.empty((m, 3), np.float32)
    v = np.empty((m, 3, 3), np.float32)
    check(lib().pcd_host_eigh3(t6.ctypes.data, m, w.ctypes.data, v.ctypes.data), "pcd_host_eigh3")
    return w, v


def host_vu_smooth(w, v, n, tau=0.3, damp=3.0):
    import numpy as np
    w = np.ascontiguousarray(w, np.float32); v = np.ascontiguousarray(v, np.float32)
    n = np.ascontiguousarray(n, np.float32)
    out = np.empty_like(n)
    check(lib().pcd_host_vu_smooth(w.ctypes.data, v.ctypes.data, n.ctypes.data, n.shape[0], float(tau), float(damp),
                                   out.ctypes.data), "pcd_host_vu_smooth")
    return out


def host_nvt_tensor(pos, n, ci, off, nbr, rho):
    """The fused kernels' NVT vote + tensor sums on the host (numpy in, (m, 6) float32 out)."""
    import numpy as np
    pos = np.ascontiguousarray(pos, np.float32); n = np.ascontiguousarray(n, np.float32)
    ci = np.ascontiguousarray(ci, np.int64); off = np.ascontiguousarray(off, np.int64)
    nbr = np.ascontiguousarray(nbr, np.int64)
    out = np.empty((len(ci), 6), np.float32)
    check(lib().pcd_host_nvt_tensor(pos.ctypes.data, n.ctypes.data, ci.ctypes.data, off.ctypes.data, nbr.ctypes.data,
                                    len(ci), float(rho), out.ctypes.data), "pcd_host_nvt_tensor")
    return out


def host_solve3(a, b):
    import numpy as np
    a = np.ascontiguousarray(a, np.float32); b = np.ascontiguousarray(b, np.float32)
    x = np.zeros_like(b)
    ok = np.zeros(b.shape[0], np.int32)
    check(lib().pcd_host_solve3(a.ctypes.data, b.ctypes.data, b.shape[0], x.ctypes.data, ok.ctypes.data),
          "pcd_host_solve3")
    return x, ok.astype(bool)


def host_inv3(a):
    """torch.linalg.inv_ex's arithmetic for 3x3 as the position steps restate it (host build): (inverse, ok)."""
    import numpy as np
    a = np.ascontiguousarray(a, np.float32)
    x = np.zeros_like(a)
    ok = np.zeros(a.shape[0], np.int32)
    check(lib().pcd_host_inv3(a.ctypes.data, a.shape[0], x.ctypes.data, ok.ctypes.data), "pcd_host_inv3")
    return x, ok.astype(bool)


def host_step_csr(kind, pos, n, edge_vectors, ci, nbr, d, alpha, delta=0.0):
    """The kernels' Denoiser.*_step on the host (dense neighbour rows nbr [m, k]): out [m, 3]."""
    import numpy as np
    pos = np.ascontiguousarray(pos, np.float32); n = np.ascontiguousarray(n, np.float32)
    ev = None if edge_vectors is None else np.ascontiguousarray(edge_vectors, np.float32)
    ci = np.ascontiguousarray(ci, np.int64); nbr = np.ascontiguousarray(nbr, np.int64)
    m, k = nbr.shape
    off = np.arange(m + 1, dtype=np.int64) * k
    out = np.empty((m, 3), np.float32)
    check(lib().pcd_host_step_csr(int(kind), pos.ctypes.data, n.ctypes.data, None if ev is None else ev.ctypes.data,
                                  ci.ctypes.data, off.ctypes.data, nbr.ctypes.data, m, float(delta), float(d),
                                  float(alpha), out.ctypes.data), "pcd_host_step_csr")
    return out


def orient_normals_mst(pos_host, n_host, a_host, b_host):
    """Host (CPU) MST orientation; tensors must be contiguous CPU f32 / int64.  Modifies n_host in place."""
    assert not pos_host.is_cuda and not n_host.is_cuda
    check(lib().pcd_orient_normals_mst(ptr(pos_host), ptr(n_host), pos_host.size(0), ptr(a_host), ptr(b_host),
                                       a_host.size(0)), "pcd_orient_normals_mst")


def orient_normals_mst_gpu(pos, n, a, b) -> torch.Tensor:
    """Device MST orientation (Borůvka + Euler tour + sign pointer jumping), bit-identical to the host version.
    Returns the oriented normals as a new device f32 tensor; the inputs are not modified."""
    p = f32(pos)
    out = f32(n).clone()
    a = i64(a).reshape(-1)
    b = i64(b).reshape(-1)
    assert p.dim() == 2 and p.size(1) == 3 and out.shape == p.shape and a.numel() == b.numel()
    check(lib().pcd_orient_normals_mst_gpu(ptr(p), ptr(out), p.size(0), ptr(a), ptr(b), a.numel(),
                                           c_void_p(stream_ptr())), "pcd_orient_normals_mst_gpu")
    return out
