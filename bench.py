"""Benchmark: Mpoints/s per denoise iteration (kNN + NVT/PCA + update) at k = 32 on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points P] [--k 32] [--k-update 8]

--gpus N > 1 launches the N ranks itself (one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set for
each) before anything touches a GPU, and refuses to run on a box with fewer than N GPUs unless --rehearse-one-gpu
puts every rank on GPU 0 (libpcd's host-callback transport instead of RCCL).  Launched by torchrun instead
(WORLD_SIZE already set), each process is one rank as it stands.

Workload (BASELINE.json configs[3], the headline): `xyzrgb_dragon.obj` is a missing blob in the reference, so
the substitute of BASELINE.md is used -- P (default 10,000,000) area-weighted samples of stanford-bunny.obj
(data/stanford_bunny_mesh.npz), isotropic Gaussian noise sigma = 0.005 x bbox diagonal, analytic face normals.
One "step" = one full iteration of Processor.denoise's loop body on device-resident data: kNN(k) against the
frozen snapshot -> NVT1 + VU smoothing -> NVT2 + classes -> flat (global reduce) / edge / corner updates.
Excluded (one-time): snapshot/grid build, initial normals, mean edge length l, data synthesis.

Multi-GPU (BASELINE configs[4]): one global cloud of N x P points, made on rank 0 (the coordinator,
the only process that holds it), is cut into N spatial slabs along its longest axis; rank 0 hands every rank its slab
+ halo over libpcd's RCCL communicator, each rank denoises its slab and exchanges halo rows with its slab neighbours
(pcd_slab_iterate: RCCL over xGMI, plus two scalar all-reduces per flat phase) -- weak scaling (P points per GPU).
torch.distributed is a gloo group for control only.  --replicas instead runs N independent P-point clouds.  The
timed region is bracketed by barrier + synchronize and the max over ranks is reported; the slab coverage check of
the timed iterations runs right after it (a thin halo re-plans and the region is timed again).

The JSON line carries `roofline` for the dominant stage (K1 = kNN + NVT1, HIP events on its launch stream),
`kernel_ms` per stage (HIP events in a replay of the timed iterations; `knn_nvt1` from the timed region itself, whose
iterations record K1's two events only), `ten_iteration_ms` (a fresh cloud through configs[3]'s 10 iterations, the dense
first anchoring included), `measured_traffic` (the rocprofv3 PMC bytes of profiles/traffic.json per iteration against
8 TB/s, null when that file was measured on another build of libpcd), `cpu_baseline` (the oracle restatement on host
cores over a bounded sample) and `parity` (the same sample through one GPU iteration: Chamfer distance to the clean
surface vs the oracle's, class agreement); the last two on rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import pcd_native as nat  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud, sample_surface  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
# what the PMC byte counts are (profiles/r3/calib_traffic.json): memory-side requests of the L2, so Infinity-Cache
# (MALL) hits count too -- an upper bound on HBM bytes, not HBM bytes
TRAFFIC_KIND = ("L2-miss bytes per launch: rocprofv3 FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE; Infinity-Cache "
                "hits included, so an upper bound on HBM traffic")


# Per-stage bound, as the rocprofv3 counters of profiles/ show it, VALU issue priced at gfx950's 2
# cycles per wave64 instruction: valu = the SIMD's VALU issue busy >= ~1/2 of the kernel, latency = waves parked on
# memory most of the time, ta = the texture addresser busy (one cycle per active lane of a gather).
STAGE_BOUND = {"anchor_test": "ta (64 row gathers a row)", "requery": "latency", "spill_search": "latency",
               "nvt1": "valu+latency", "nvt2": "latency+valu", "flat_phase": "latency", "edge_phase": "latency",
               "corner_phase": "latency", "finish": "-"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def knn_cap(k):
    """Register list size the fused kernel is instantiated with (pcd_denoiser_iterate)."""
    return 8 if k <= 8 else 16 if k <= 16 else 32 if k <= 32 else 64


def k1_kernels(k, ku, seeding, anchoring):
    """Kernels of the K1 stage (kNN + NVT1) as pcd_denoiser_iterate launches them in a timed (seeded) step."""
    c = knn_cap(max(k, ku))
    unit = "true"    # k_nvt1<C, UNIT>: every timed iteration runs on the loop's own unit normals
    if seeding and anchoring and c <= 32:
        return [f"k_knn_anchor<{c}, {2 * c}>", "k_compact_fail", f"k_knn_requery<{2 * c}, 64>",
                f"k_knn_redo_wave<{2 * c}, false>", f"k_nvt1<{c}, {unit}>"]
    return [f"k_knn_nvt1<{c}, {'true' if seeding else 'false'}>"]


def b_alg_iteration(k, ku):
    """Algorithmic bytes / point / iteration: 148 + 72k + 60k_u."""
    return 148 + 72 * k + 60 * ku


def b_alg_knn_nvt1(k):
    """K1 stage (kNN + NVT1), SURVEY.md §8(d): kNN 12 (query) + 12k (winners' xyz) + 4k (list write) and NVT1 4k (list)
    + 12 (own v) + 24k (v_j, n_j) + 12 (own n) + 12 (f_n write) = 48 + 44k (1,456 B at k = 32)."""
    return (12 + 12 * k + 4 * k) + (4 * k + 12 + 24 * k + 12 + 12)


def make_cloud(n, seed, dev, sigma_frac=0.005, clean=False):
    m = np.load(os.path.join(ROOT, "data", "stanford_bunny_mesh.npz"))
    v = torch.from_numpy(m["v"]).to(dev)
    f = torch.from_numpy(m["f"].astype(np.int64)).to(dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    surf, nrm = sample_surface(v, f, n, generator=g)
    diag = float((v.max(0).values - v.min(0).values).norm())
    pos = surf + sigma_frac * diag * torch.randn(surf.shape, generator=g, device=dev)
    if clean:
        return pos.contiguous(), nrm.contiguous(), diag, surf.contiguous()
    return pos.contiguous(), nrm.contiguous(), diag


def cpu_baseline(k, ku, sample_points, dev, seed=99):
    """The oracle (numpy/scipy restatement of the reference, cKDTree workers=1) for one iteration on a bounded sample,
    and the same sample through one fused GPU iteration: (cpu_baseline, parity) blocks of the JSON line."""
    from oracle import pcd_oracle as O
    # the host share this process may use: affinity mask, capped by OMP_NUM_THREADS (16 on the GPU box)
    threads = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(threads)
    pos, nrm, _, surf = make_cloud(sample_points, seed, torch.device("cpu"), clean=True)
    pos, nrm = pos.numpy(), nrm.numpy()
    knn = O.FrozenKNN(pos)
    d = 2 * O.mean_edge_length(pos, knn)
    t0 = time.perf_counter()
    rpos, _, rcls = O.denoise_iteration(pos, nrm, knn, d, k, ku)
    dt = time.perf_counter() - t0
    base = {"value": round(sample_points / dt / 1e6, 5), "unit": "Mpoints/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"1 iteration of the oracle restatement on {sample_points:,} bunny-sampled points "
                      f"(k={k}, k_u={ku}), scipy cKDTree workers=1, torch intra-op threads={threads}, "
                      f"{dt:.2f} s"}
    # parity on the same sample: one fused GPU iteration, Chamfer distance to the noiseless surface samples
    from Pointcloud.Modules.Utils import TorchUtils
    proc = Processor(Pointcloud(torch.from_numpy(pos).to(dev), torch.from_numpy(nrm).to(dev)), k_hint=k)
    fused = proc._fused_for(max(k, ku))
    fused.load(proc.graph.pos, proc.graph.n)
    fused.iterate(nat.make_params(k=k, k_update=ku, d=d), 1)
    gp = torch.empty((sample_points, 3), device=dev)
    gc = torch.empty(sample_points, dtype=torch.int64, device=dev)
    fused.store(gp, None, gc)
    gt = surf.to(dev)
    cd_gpu = float(TorchUtils.ChamferDistance(gt, gp).mean())
    cd_ref = float(TorchUtils.ChamferDistance(gt, torch.from_numpy(rpos).to(dev)).mean())
    cd_in = float(TorchUtils.ChamferDistance(gt, torch.from_numpy(pos).to(dev)).mean())
    parity = {"sample": f"the cpu_baseline sample ({sample_points:,} points), 1 iteration, Chamfer distance to the "
                        f"noiseless surface samples", "cd_noisy": cd_in, "cd_oracle": cd_ref, "cd_gpu": cd_gpu,
              "cd_delta_rel": abs(cd_gpu - cd_ref) / cd_ref,
              "class_agreement": float((gc.cpu().numpy() == rcls).mean())}
    return base, parity


def mesh_bench(dev, cpu):
    """Mesh.updateVertices (H18, PatchGeneration/Modules/Mesh.py:377-418): per-sweep time of the fp64 kernel (the
    reference's arithmetic) and the fp32 kernel on the bunny mesh (the reference publishes 0.591 s/iteration for
    Algorithm 3 on an unshipped mesh, Vertex_updating.ipynb:300) and on a 2048 x 2048 height-field grid (4.2M vertices)
    for the fp32 roofline at 32 + 64 deg B/vertex; adjacency built on the device.  Per-sweep = (t(16
    sweeps) - t(1 sweep)) / 15 by host wall clock around synchronised calls (excludes the fp32 path's row repacking)."""
    m = np.load(os.path.join(ROOT, "data", "stanford_bunny_mesh.npz"))
    out = {"reference_s_per_iteration": 0.591, "reference_source": "Vertex_updating.ipynb:300 (Algorithm 3 = "
           "Mesh.updateVertices, author's CPU, mesh example_object.obj not shipped)"}

    def per_sweep(v, f, fn, vf, ni, fp32):
        fun = nat.mesh_update_f32 if fp32 else nat.mesh_update
        ts = {}
        for k in (1, 16):
            best = float("inf")
            for _ in range(3):
                w = v.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fun(w, f, fn, vf, ni, k)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            ts[k] = best
        return (ts[16] - ts[1]) / 15

    def setup(v, f, fp32):
        it, ft = (torch.int32, torch.float32) if fp32 else (torch.int64, torch.float64)
        vd = v.to(dev, ft).contiguous()
        fd = f.to(dev, it).contiguous()
        a, b, c = vd[fd[:, 0].long()], vd[fd[:, 1].long()], vd[fd[:, 2].long()]
        cr = torch.cross(b - a, c - b, dim=1)
        fn = (cr / cr.norm(dim=1, keepdim=True).clamp(min=1e-30)).contiguous()
        vf, ni = nat.mesh_vta(fd, vd.size(0), out_dtype=it)
        return vd, fd, fn, vf, ni

    bv, bf = torch.from_numpy(m["v"].astype(np.float64)), torch.from_numpy(m["f"].astype(np.int64))
    out["bunny"] = {"vertices": int(bv.size(0)), "faces": int(bf.size(0)),
                    "fp64_ms_per_iteration": round(per_sweep(*setup(bv, bf, False), False) * 1e3, 4),
                    "fp32_ms_per_iteration": round(per_sweep(*setup(bv, bf, True), True) * 1e3, 4)}
    # a 2048 x 2048 grid mesh (two triangles per quad) over a smooth height field, on the device
    n = 2048
    ys, xs = torch.meshgrid(torch.linspace(0, 1, n, device=dev), torch.linspace(0, 1, n, device=dev), indexing="ij")
    gv = torch.stack([xs, ys, 0.05 * torch.sin(12 * xs) * torch.cos(9 * ys)], -1).reshape(-1, 3)
    q = torch.arange((n - 1) * (n - 1), device=dev)
    r0 = (q // (n - 1)) * n + q % (n - 1)
    gf = torch.cat([torch.stack([r0, r0 + 1, r0 + n], 1), torch.stack([r0 + 1, r0 + n + 1, r0 + n], 1)])
    vd, fd, fn, vf, ni = setup(gv, gf, True)
    t = per_sweep(vd, fd, fn, vf, ni, True)
    nv, nf = vd.size(0), fd.size(0)
    deg = 3 * nf / nv
    gather = (32 + 64 * deg) * nv            # every gathered attribute counted per use
    # HBM bytes when every array is streamed once (the re-reads of shared faces / corner rows are L2 hits): vertex
    # rows in and out (16 + 16), NI 4, VF 4 deg, face normals and corner ids 16 + 16 per face
    unique = (16 + 16 + 4 + 4 * deg) * nv + (16 + 16) * nf
    out["grid_fp32"] = {"vertices": int(nv), "faces": int(nf), "ms_per_iteration": round(t * 1e3, 4),
                        "roofline": {"bound": "hbm", "bytes_per_vertex": round(unique / nv, 1),
                                     "achieved": round(unique / t / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(unique / t / 1e9 / HBM_PEAK_GBS, 4),
                                     "model": "each array streamed once (vertex rows in + out, NI, VF, face normals, "
                                              "face corner ids); the per-use re-reads hit L2"},
                        "gather_model": {"alg_bytes_per_vertex": round(32 + 64 * deg, 1),
                                         "achieved": round(gather / t / 1e9, 2), "unit": "GB/s",
                                         "note": "SURVEY §8(d)'s 32 + 64 deg B/vertex counts every gathered "
                                                 "attribute per use, so it exceeds HBM peak once L2 serves the reuse"}}
    if cpu:
        from oracle import pcd_oracle as O
        vn, fn_ = m["v"].astype(np.float64), m["f"].astype(np.int64)
        cr = np.cross(vn[fn_[:, 1]] - vn[fn_[:, 0]], vn[fn_[:, 2]] - vn[fn_[:, 1]])
        nrm = cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)
        t0 = time.perf_counter()
        O.mesh_update(vn, fn_, nrm, k=3)
        out["bunny"]["cpu_oracle_s_per_iteration"] = round((time.perf_counter() - t0) / 3, 4)
    return out


def cpsd_alg_bytes(m, ku=8):
    """Algorithmic bytes / point / iteration of the fused CPSD driver (pcd_cpsd_iterate), SURVEY §8(d)'s convention
    (every neighbour attribute read counted per use, f32 values, int32 indices), m = mean radius members:
      kNN(k_u) lists       12 + 12 k_u + 4 k_u
      radius NVT + VU      12 (own pos) + 12 m (member xyz) + 12 m (n_j) + 12 (own n) + 12 (f_n) + 4 m (member rows)
      PVT + VU features    4 m (rows) + 24 (own pos, f_n) + 3 x 12 m (f_n_j: the vote, and again in the two sums)
                           + 2 x 12 m (v_j: centroid and covariance) + 13 (class, edge vector)
      phases (Jacobi)      flat reduce 2 (4 + 16 k_u) + update 4 + 4 k_u + 36 + 24 k_u + 12 (+ 16: the global clamp's orig)"""
    knn = 12 + 16 * ku
    nvt = 36 + 28 * m
    pvt = 37 + 64 * m
    phases = 2 * (4 + 16 * ku) + 4 + 28 * ku + 48 + 16
    return knn + nvt + pvt + phases


def cpsd_bench(dev, cpu, sizes=(50_000, 1_000_000), iterations=50):
    """The CPSD ("Martin") 50-iteration driver (PostProcessing.ipynb:1041-1062, Processor.cpsdDenoise -> one
    pcd_cpsd_iterate call) on bunny-sampled clouds: seconds per iteration against the reference's 1.13 s/it on the
    50k-point Stitch_guitar (PostProcessing.ipynb:1015, author's CPU), and at 1M points a roofline on
    cpsd_alg_bytes."""
    out = {"reference_s_per_iteration": 1.13, "reference_source": "PostProcessing.ipynb:1015 (50k-point Stitch_guitar, "
           "author's CPU)", "iterations": iterations}
    for points in sizes:
        pos, nrm, _ = make_cloud(points, 4, dev)
        proc = Processor(Pointcloud(pos.clone(), nrm.clone()), k_hint=16)
        d = 2 * float(proc.meanEdgeLength())
        m = float(proc.selector.getPointsInRangeSelection(d).slices.diff().float().mean())
        proc.cpsdDenoise(iterations=2, d=d)                  # warm-up (allocations, list slots, kernels)
        proc.pointcloud.v.copy_(pos)
        proc.graph.n = nrm.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        proc.cpsdDenoise(iterations=iterations, d=d)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iterations
        row = {"points": points, "s_per_iteration": round(dt, 6), "mean_members": round(m, 2)}
        if points == 50_000:
            row["speedup_vs_reference"] = round(1.13 / dt, 1)
            if cpu:
                from oracle import pcd_oracle as O
                p0, n0 = pos.cpu().numpy(), nrm.cpu().numpy()
                knn = O.FrozenKNN(p0)
                t1 = time.perf_counter()
                O.cpsd_iteration(p0, p0, n0, p0, knn, d)
                row["cpu_oracle_s_per_iteration"] = round(time.perf_counter() - t1, 4)
        b = cpsd_alg_bytes(m) * points
        row["roofline"] = {"bound": "valu+latency", "alg_bytes_per_point": round(cpsd_alg_bytes(m), 1),
                           "achieved": round(b / dt / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(b / dt / 1e9 / HBM_PEAK_GBS, 4)}
        out[f"n{points // 1000}k"] = row
    if "n50k" in out:          # (the round-3 keys, kept)
        out["points"] = 50_000
        out["s_per_iteration"] = out["n50k"]["s_per_iteration"]
        out["speedup_vs_reference"] = out["n50k"].get("speedup_vs_reference")
    return out


def slab_world1_bench(pos, nrm, params, args, fused_ms):
    """The multi-GPU driver (pcd_slab.SlabDenoiser: one pcd_slab_iterate call per iteration, the coverage check and
    checkpoint every 10 iterations, as the N-GPU bench runs it) at one rank on the headline workload, timed like the
    main line (warm-up, then the steps between synchronisations): its overhead over the fused loop at N = 1."""
    from pcd_slab import LocalTransport, SlabDenoiser
    sd = SlabDenoiser(pos, nrm, max(args.k, args.k_update), transport=LocalTransport(), seeding=args.seeding,
                      check_every=10)
    for _ in range(args.warmup):
        sd.iterate(params, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sd.iterate(params, 1)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    sd.check()
    stages = sd.iterate_timed(params)
    out = {"ms_per_step": round(ms, 4), "ratio_to_fused_loop": round(ms / fused_ms, 4),
           "stage_ms": {k: round(v, 4) for k, v in stages.items()},
           "note": "SlabDenoiser + LocalTransport, one pcd_slab_iterate call per iteration, coverage check and "
                   "checkpoint every 10 iterations inside the timed steps"}
    del sd
    torch.cuda.empty_cache()
    return out


def n1_point(args, dev):
    """The single-GPU fused loop on args.points points (seed 2, the N = 1 bench's cloud): warm-up, then the timed
    steps between synchronisations."""
    pos, nrm, _ = make_cloud(args.points, 2, dev)
    proc = Processor(Pointcloud(pos, nrm), k_hint=args.k)
    d = 2 * float(proc.meanEdgeLength())
    fused = proc._fused_for(max(args.k, args.k_update))
    fused.load(proc.graph.pos, proc.graph.n)
    params = nat.make_params(k=args.k, k_update=args.k_update, d=d)
    fused.iterate(params, args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fused.iterate(params, args.steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    fused.check()
    out = {"points": args.points, "ms_per_step": round(ms, 4), "value": round(args.points / ms / 1e3, 3),
           "unit": "Mpoints/s", "note": "rank 0 alone, single-GPU fused loop, same per-GPU point count, after the "
                                        "slab run (its state still resident)"}
    del fused, proc
    torch.cuda.empty_cache()
    return out


def measured_traffic(points, k, ms_per_step):
    """HBM bytes per iteration from profiles/traffic.json (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch, the
    gfx950 correction of MI355X_MICROARCH.md), summed over the iteration's kernels, against 8 TB/s."""
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(tfile):
        return None
    try:
        tj = json.load(open(tfile))
    except (OSError, ValueError):
        return None
    if tj.get("points") != points or tj.get("k") != k or "per_iteration_bytes" not in tj:
        return None
    if tj.get("build_id") != nat.build_id():
        return {"bytes_per_iteration": None, "frac": None, "traffic_build": tj.get("build_id"),
                "lib_build": nat.build_id(), "note": "profiles/traffic.json was measured on another build of libpcd"}
    b = float(tj["per_iteration_bytes"])
    return {"bytes_per_iteration": b, "traffic_build": tj["build_id"],
            "achieved": round(b / (ms_per_step / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(b / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "kind": TRAFFIC_KIND,
            "source": tj.get("source", "profiles/traffic.json")}


def progress(msg: str):
    """A progress line on stderr (rank 0 of a multi-rank run): long set-ups stay visibly alive."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, rehearse: bool) -> int:
    """--gpus N > 1 without a launcher: start N rank processes of this script (nothing here has touched a GPU) and
    return the first non-zero exit status (the others are then stopped), else 0."""
    import subprocess
    have = torch.cuda.device_count()          # (counting devices does not initialise one)
    if have < n and not rehearse:
        print(f"bench.py: --gpus {n} needs {n} GPUs, this box has {have} (--rehearse-one-gpu puts every rank on "
              f"GPU 0 over libpcd's host transport)", file=sys.stderr, flush=True)
        return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, alive = 0, set(range(n))
    while alive:
        for r in sorted(alive):
            code = procs[r].poll()
            if code is None:
                continue
            alive.discard(r)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.1)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--k-update", type=int, default=8)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-seeding", dest="seeding", action="store_false",
                    help="run every kNN search unseeded (the seeded search is the default; identical results)")
    ap.add_argument("--no-anchoring", dest="anchoring", action="store_false",
                    help="seeded searches without anchors (capped grid search every iteration; identical results)")
    ap.add_argument("--profile-steps", type=int, default=5,
                    help="slab mode: extra per-stage timed iterations after the timed region (torch events)")
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: independent clouds per rank instead of spatial slabs of one global cloud")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1 slabs: one global cloud of --points in total (strong scaling, BASELINE configs[4] "
                         "asks for 80M), instead of --points per GPU")
    ap.add_argument("--long-run", type=int, default=100,
                    help="continue the ten-iteration cloud to this iteration, per-iteration times (long_run)")
    ap.add_argument("--no-extras", dest="extras", action="store_false",
                    help="skip the mesh-update and CPSD-driver measurements (mesh_update, cpsd)")
    ap.add_argument("--no-rebalance", dest="rebalance", action="store_false",
                    help="slab mode: keep the equal-count cut (default: re-cut by class cost after warm-up 2)")
    ap.add_argument("--no-slab1", dest="slab1", action="store_false",
                    help="skip the slab_world1 block (the multi-GPU driver at one rank on the same workload)")
    ap.add_argument("--no-ten", dest="ten", action="store_false",
                    help="skip the ten_iteration_ms measurement (fresh cloud, 10 iterations incl. the first)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1: every rank on GPU 0, libpcd's host-callback transport over gloo instead of RCCL "
                         "(a rehearsal of the multi-GPU path on a one-GPU box; not a scaling number)")
    ap.add_argument("--no-n1", dest="n1", action="store_false",
                    help="N > 1: skip the N = 1 comparison point (rank 0 alone, the same per-GPU workload)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, args.rehearse_one_gpu))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr, flush=True)
    if world > 1 and not args.rehearse_one_gpu and torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks need {world} GPUs, this box has {torch.cuda.device_count()}",
              file=sys.stderr, flush=True)
        sys.exit(2)
    local = 0 if args.rehearse_one_gpu else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # control plane only (plan scalars, verdicts, the timing max); the data plane is libpcd's communicator
        dist.init_process_group("gloo")
    mode = "single" if world == 1 else ("replicas" if args.replicas else "slab")

    if mode == "slab":
        # one global cloud of world x P points, made and held by rank 0 only (the coordinator), cut into spatial slabs
        # with a halo; d = 2 l (Processor.py:120-121) likewise on rank 0 -- the other ranks never see the whole cloud
        from pcd_slab import SlabDenoiser, TorchTransport
        total = args.points if args.strong else args.points * world
        pos = nrm = None
        dt = torch.zeros(1, dtype=torch.float64)
        if rank == 0:
            progress(f"slab mode: sampling the {total:,}-point cloud on rank 0")
            pos, nrm, diag = make_cloud(total, 3, dev)
            dt[0] = 2 * float(Processor(Pointcloud(pos), k_hint=args.k).meanEdgeLength())
            progress("d = 2 l computed; planning the slabs")
        dist.broadcast(dt, 0)
        d = float(dt)
        # coverage checked every 10 iterations (a thin halo re-plans and replays, pcd_slab); slabs re-cut by class
        # cost after the first warm-up iteration (rebalance), so the timed region runs on the balanced plan.  The
        # first plan covers that one iteration (its k-balls at the snapshot); the re-cut prices the drift measured
        # over it for every iteration that follows (cut_spheres), so the run needs no coverage re-plan.
        reb = args.rebalance and args.warmup >= 2
        tr = TorchTransport(rccl=not args.rehearse_one_gpu)
        sd = SlabDenoiser(pos, nrm, max(args.k, args.k_update), transport=tr, seeding=args.seeding, check_every=10,
                          step_bound=d, horizon=1 if reb else args.warmup + args.steps)
        progress(f"slabs handed out (halo {sd.halo:.4g}); warm-up")
        del pos, nrm
        torch.cuda.empty_cache()
        params = nat.make_params(k=args.k, k_update=args.k_update, d=d)
        step = lambda: sd.iterate(params, 1)  # noqa: E731
    else:
        pos, nrm, diag, surf = make_cloud(args.points, 2 + rank, dev, clean=True)
        pc = Pointcloud(pos, nrm)
        proc = Processor(pc, k_hint=args.k)
        d = 2 * float(proc.meanEdgeLength())
        fused = proc._fused_for(max(args.k, args.k_update))
        fused.load(proc.graph.pos, proc.graph.n)
        fused.set_seeding(args.seeding)
        fused.set_anchoring(args.anchoring)
        params = nat.make_params(k=args.k, k_update=args.k_update, d=d)
        step = lambda: fused.iterate(params, 1)  # noqa: E731

    first_ms = None
    for w in range(args.warmup):
        if w == 0:                 # iteration 1 builds every anchor (dense search): reported on its own
            torch.cuda.synchronize()
            tf = time.perf_counter()
            step()
            torch.cuda.synchronize()
            first_ms = (time.perf_counter() - tf) * 1e3
        else:
            step()
        if mode == "slab" and reb and w == 0:
            # cost-weighted cut from this iteration's classes (the next iteration re-anchors), sized for the rest
            sd.rebalance(horizon=args.warmup - 1 + args.steps)
            progress("re-cut by class cost")
        if mode == "slab":
            progress(f"warm-up iteration {w + 1}/{args.warmup}")
    if mode != "slab":
        # the K1 stage's two HIP events on the launch stream, every timed iteration (the roofline's kernel time); the
        # other stages' events (~4 us each, ~0.04 ms an iteration) are recorded in a replay of the same iterations
        fused.set_timing(2)

    def timed_region():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return el

    if mode == "slab":
        progress("timed region")
        # the timed iterations carry no coverage check (a host sync + an all-reduce): it runs right after them, and a
        # thin halo there (re-planned and replayed) sends the region round again on the widened plan
        every = sd.check_every
        for _attempt in range(3):
            sd.checkpoint()
            sd.check_every = args.steps + 1
            replans = sd.replans
            rs0 = sd.e.readset_stats() if hasattr(sd.e, "readset_stats") else (0, 0, 0)
            elapsed = timed_region()
            rs1 = sd.e.readset_stats() if hasattr(sd.e, "readset_stats") else (0, 0, 0)
            sd.verify()
            sd.check_every = every
            if sd.replans == replans:
                break
    else:
        elapsed = timed_region()
    ms_per_step = elapsed / args.steps * 1e3
    total_points = args.points if (mode == "slab" and args.strong) else args.points * world
    value = total_points / (ms_per_step / 1e3) / 1e6

    # per-kernel timing (HIP events on the launch stream), outside the timed region
    kernel_ms, knn_ms = {}, float("nan")
    xchg = None
    if mode == "slab":
        sd.check()      # exactness: no k-ball left its rank's slab + halo
        if sd.native:
            # one halo refresh on its own (FIELD_POS: pack -> libpcd comm -> unpack), every rank at once: the median of
            # 5, max over the ranks (an idempotent refresh between iterations)
            xs = []
            for _ in range(5):
                torch.cuda.synchronize()
                dist.barrier()
                tx = time.perf_counter()
                sd.e.fused.halo_exchange(sd.comm, nat.FIELD_POS)
                torch.cuda.synchronize()
                xs.append((time.perf_counter() - tx) * 1e3)
            xt = torch.tensor([float(np.median(xs))], dtype=torch.float64)
            dist.all_reduce(xt, op=dist.ReduceOp.MAX)
            xchg = float(xt)
        ks = [sd.iterate_timed(params) for _ in range(args.profile_steps)]
        if ks:
            kernel_ms = {key: round(float(np.mean([x[key] for x in ks])), 4) for key in ks[0]}
            knn_ms = kernel_ms["knn_nvt1"]
    else:
        k1 = fused.timing()         # K1's ms, averaged over exactly the timed iterations
        fused.set_timing(False)
        fused.check()               # device error word: invalid list entries would fail the bench here
        if k1:
            knn_ms = float(k1[0])
        # the per-stage split: the same cloud's same iterations replayed (reloaded, anchors reset: the iterations are
        # deterministic, so iterations 1..warmup untimed and the next `steps` with every stage's events), outside
        # the timed region
        fused.load(proc.graph.pos, proc.graph.n)
        fused.reset_seed()
        fused.iterate(params, args.warmup)
        fused.set_timing(True)
        fused.iterate(params, args.steps)
        slots = fused.timing()
        fused.set_timing(False)
        fused.check()
        if slots:
            names = nat.FusedDenoiser.TIMING_SLOTS
            kernel_ms = {names[i]: round(float(slots[i]), 4) for i in range(min(len(slots), len(names)))}
            kernel_ms["knn_nvt1_replay"] = round(float(sum(slots[:4])), 4)
        if knn_ms == knn_ms:
            kernel_ms["knn_nvt1"] = round(knn_ms, 4)
    ten_ms = None
    if mode != "slab" and args.ten:
        # configs[3] as written: a fresh cloud (no anchors yet) through 10 iterations, the dense first one included
        fused.load(proc.graph.pos, proc.graph.n)
        fused.reset_seed()
        torch.cuda.synchronize()
        t10 = time.perf_counter()
        fused.iterate(params, 10)
        torch.cuda.synchronize()
        ten_ms = (time.perf_counter() - t10) * 1e3
        fused.check()
    long_run = None
    chamfer = None
    if mode != "slab" and args.ten:
        # the Chamfer distance of the 10-iteration result to the clean surface samples, at full size on the GPU
        # (pcd_nn_dist: two nearest-neighbour passes over Morton-ordered queries), timed outside every bench region
        from Pointcloud.Modules.Utils import TorchUtils
        den = torch.empty_like(surf)
        fused.store(den, torch.empty_like(surf))
        torch.cuda.synchronize()
        tc = time.perf_counter()
        cd_den = float(TorchUtils.ChamferDistance(surf, den).mean())
        torch.cuda.synchronize()
        cd_ms = (time.perf_counter() - tc) * 1e3
        cd_in = float(TorchUtils.ChamferDistance(surf, pos).mean())
        chamfer = {"points": args.points, "ms": round(cd_ms, 3), "cd_noisy": cd_in, "cd_10_iterations": cd_den}
        # the long run (north_star: "iterated to convergence"): the same cloud on to iteration 100, per-iteration
        # HIP-event time and re-anchored rows (the re-anchoring rate peaks near iteration 30)
        fused.set_timing(True)
        per_it, redo = {}, {}
        for it in range(11, args.long_run + 1):
            fused.iterate(params, 1)
            per_it[it] = float(sum(fused.timing()))
            redo[it] = fused.redo_rows()
        fused.set_timing(False)
        fused.check()
        if per_it:
            at = [a for a in (25, 50, 75, 100) if a in per_it]
            long_run = {"iterations": args.long_run, "ms_at": {a: round(per_it[a], 4) for a in at},
                        "redo_pct_at": {a: round(100 * redo[a] / args.points, 3) for a in at},
                        "max_ms": round(max(per_it.values()), 4),
                        "max_at": max(per_it, key=per_it.get),
                        "mean_ms_last_20": round(float(np.mean([per_it[a] for a in sorted(per_it)[-20:]])), 4)}

    k1_points = sd.owned_global.numel() if mode == "slab" else args.points
    k1_bytes = b_alg_knn_nvt1(args.k) * k1_points
    achieved = k1_bytes / (knn_ms / 1e3) / 1e9 if knn_ms == knn_ms else None
    k1_names = k1_kernels(args.k, args.k_update, args.seeding, args.anchoring)
    traffic, traffic_build = None, None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile) and mode != "slab":
        try:
            tj = json.load(open(tfile))
            traffic_build = tj.get("build_id")
            if tj.get("points") == args.points and tj.get("k") == args.k and tj.get("build_id") == nat.build_id():
                per = [tj["kernels"][nm][0]["hbm_bytes_per_launch"] for nm in k1_names if nm in tj["kernels"]]
                traffic = float(sum(per)) if per else None
        except Exception:
            traffic = None
    iter_alg = b_alg_iteration(args.k, args.k_update) * args.points
    out = {
        "metric": "Mpoints/sec per denoise iteration (kNN+PCA+update), k=32, 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "Mpoints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if (mode == "slab" and args.strong) else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: bunny-sampled surface + Gaussian noise (sigma=0.005*bbox), analytic normals, "
                + ("one global cloud (seed 3) cut into spatial slabs" if mode == "slab" else "seed 2+rank"),
        "config": {"workload": ("configs[4]: synthetic %dM-point bunny-sampled surface, spatial slabs with RCCL halo"
                                % (total_points // 1_000_000) if mode == "slab" else
                                "configs[3] headline substitute: 10M-pt bunny-sampled cloud (xyzrgb_dragon.obj is "
                                "a missing blob)" if args.points == 10_000_000 else
                                "NOT the headline: %.4gM-pt bunny-sampled cloud per GPU" % (args.points / 1e6))
                               + ", k=%d, k_u=%d, 1 iteration per step" % (args.k, args.k_update),
                   "points_per_gpu": total_points // world, "k": args.k, "k_update": args.k_update,
                   "global_points": total_points,
                   "parallelism": {"single": "single", "replicas": f"replicas x{world}",
                                   "slab": f"spatial slabs x{world}"}[mode]},
        "iterations_per_sec": round(1e3 / ms_per_step, 2),
        "first_iteration_ms": round(first_ms, 3) if first_ms is not None else None,
        "ten_iteration_ms": round(ten_ms, 3) if ten_ms is not None else None,
        "iter_ms_at_100": long_run["ms_at"].get(100) if long_run else None,
        "long_run": long_run,
        "chamfer": chamfer,
        "kernel_ms": kernel_ms,
        "stage_bound": STAGE_BOUND if mode != "slab" else None,
        "iteration_roofline": {"bound": "hbm", "alg_bytes_per_point": b_alg_iteration(args.k, args.k_update),
                               "achieved": round(iter_alg / (ms_per_step / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s",
                               "frac": round(iter_alg / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
        "measured_traffic": measured_traffic(args.points, args.k, ms_per_step) if mode != "slab" else None,
        "roofline": {"kernel": "K1 stage (kNN + NVT1): " + " + ".join(k1_names), "bound": "latency+ta+valu",
                     "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "traffic_kind": TRAFFIC_KIND, "traffic_build": traffic_build,
                     "measured_frac": (round(traffic / (knn_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                                       if traffic and knn_ms == knn_ms else None),
                     "alg_bytes_per_launch": k1_bytes, "avg_launch_ms": round(knn_ms, 4)},
        "bound_statement": ("every per-iteration kernel is VALU- or memory-latency-bound (SQ counters, DESIGN.md §3): "
                            "the iteration moves ~0.28 of the 8 TB/s HBM peak by the PMC counters; `frac` is the "
                            "SURVEY §8(d) algorithmic-bytes model (each neighbour attribute read counted per use, "
                            "most of them served by LDS windows and L2), `measured_frac` the counted bytes"),
    }
    out["lib_build"] = nat.build_id()
    if out["measured_traffic"] and out["measured_traffic"].get("frac") is not None:
        out["iteration_roofline"]["measured_frac"] = out["measured_traffic"]["frac"]
    if mode == "slab":
        info = sd.comm.info()
        counts = torch.tensor([sd.owned_global.numel(), sd.halo_points], dtype=torch.int64)
        allc = [torch.zeros_like(counts) for _ in range(world)]
        dist.all_gather(allc, counts)
        # halo traffic with every held halo row refreshed once per exchange -- f_n after K1, then the positions
        # after each Gauss-Seidel phase (once per iteration in the Jacobi mode) -- as 12-byte rows on the RCCL path
        n_x = 1 + (1 if params.jacobi else params.nphases)
        xb_all = [int(c[1]) * 12 * n_x for c in allc]
        # the read-set exchange (pcd_denoiser_set_readset, the default): per iteration only the halo rows some own
        # list reads -- position + normal with the K1 refresh (24 B), f_n (12 B), positions after every phase but
        # the last (12 B each) -- plus one mask bit per held halo row; rows averaged over the timed iterations
        if rs1[0] < rs0[0]:          # (a re-plan inside the region: a new engine, its stats restarted)
            rs0 = (0, 0, 0)
        its = rs1[0] - rs0[0]
        rd = torch.tensor([(rs1[2] - rs0[2]) / its if its else -1.0], dtype=torch.float64)
        alld = [torch.zeros_like(rd) for _ in range(world)]
        dist.all_gather(alld, rd)
        read_rows = [float(x) for x in alld]
        per_row = 24 + 12 + (0 if params.jacobi else 12 * (params.nphases - 1))
        if its:
            xb = [int(r * per_row + int(c[1]) / 8) for r, c in zip(read_rows, allc)]
        else:
            xb = xb_all
        out["slab"] = {"world": info["world"], "transport": info["transport"],
                       "owned_rows": [int(c[0]) for c in allc], "halo_rows": [int(c[1]) for c in allc],
                       "read_rows_per_iteration": [round(r, 1) for r in read_rows] if its else None,
                       # held = the snapshot rows a rank keeps for its kNN (sized for the planned drift); moved = the
                       # rows the read-set exchange refreshes per iteration (what the halo costs per iteration)
                       "halo_rows_held_max": max(int(c[1]) for c in allc),
                       "halo_rows_moved_per_iteration_max": round(max(read_rows), 1) if its else None,
                       "readset": bool(its),
                       "halo": sd.halo, "replans": sd.replans, "replan_log": sd.replan_log,
                       "exchanges_per_iteration": (1 + 1 + (0 if params.jacobi else params.nphases - 1)) if its
                       else n_x,
                       "exchange_bytes_per_iteration": sum(xb),
                       "exchange_bytes_per_iteration_max_rank": max(xb),
                       "exchange_bytes_per_iteration_all_halo_rows": sum(xb_all),
                       "exchange_ms": None if xchg is None else round(xchg, 4),
                       "exchange_ms_kind": "one FIELD_POS refresh of every held halo row (pcd_halo_exchange), "
                                           "median of 5, max over ranks",
                       "rehearsal_one_gpu": bool(args.rehearse_one_gpu),
                       "note": ("every rank on GPU 0 over libpcd's host transport: a rehearsal, not a scaling number"
                                if args.rehearse_one_gpu else
                                "one GPU per rank, halo rows and the flat phase's scalars over libpcd's RCCL "
                                "communicator (xGMI); gloo carries control only")}
        if args.n1:
            # the N = 1 comparison point: rank 0 alone runs the single-GPU fused loop on the per-GPU workload (the
            # N = 1 bench's cloud, seed 2), timed like the main region; the other ranks wait
            if rank == 0:
                out["n1"] = n1_point(args, dev)
            dist.barrier()
    if rank == 0 and world == 1 and args.slab1:
        out["slab_world1"] = slab_world1_bench(pos, nrm, params, args, ms_per_step)
    if rank == 0 and world == 1 and args.extras:
        out["mesh_update"] = mesh_bench(dev, not args.no_cpu_baseline)
        out["cpsd"] = cpsd_bench(dev, not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["parity"] = cpu_baseline(args.k, args.k_update, args.cpu_sample, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if mode == "slab":
        del sd
        tr.close()             # libpcd's RCCL communicator, torn down by every rank at this point
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
