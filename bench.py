"""Benchmark: Mpoints/s per denoise iteration (kNN + NVT/PCA + update) at k = 32 on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points P] [--k 32] [--k-update 8]
    torchrun --nproc-per-node N ... bench.py --gpus N          (one process per GPU; weak scaling)

Workload (BASELINE.json configs[3], the headline): `xyzrgb_dragon.obj` is a missing blob in the reference, so
the substitute of BASELINE.md is used -- P (default 10,000,000) area-weighted samples of stanford-bunny.obj
(data/stanford_bunny_mesh.npz), isotropic Gaussian noise sigma = 0.005 x bbox diagonal, analytic face normals.
One "step" = one full iteration of Processor.denoise's loop body on device-resident data: kNN(k) against the
frozen snapshot -> NVT1 + VU smoothing -> NVT2 + classes -> flat (global reduce) / edge / corner updates.
Excluded (one-time): snapshot/grid build, initial normals, mean edge length l, data synthesis.

Multi-GPU (BASELINE configs[4]): one global cloud of N x P points is cut into N spatial slabs
along its longest axis; each rank denoises its slab and exchanges halo state with its slab neighbours over RCCL
(pcd_slab), plus two scalar all-reduces per flat phase -- weak scaling (P points per GPU).  --replicas instead
runs N independent P-point clouds.  The timed region is bracketed by barrier + synchronize and the max over
ranks is reported.

The JSON line carries `roofline` for the dominant stage (K1 = kNN + NVT1, HIP events on its launch stream),
`kernel_ms` per stage (HIP events), `ten_iteration_ms` (a fresh cloud through configs[3]'s 10 iterations, the dense
first anchoring included), `measured_traffic` (the rocprofv3 PMC bytes of profiles/traffic.json per iteration against
8 TB/s), `cpu_baseline` (the oracle restatement on host cores over a bounded sample) and `parity` (the same sample
through one GPU iteration: Chamfer distance to the clean surface vs the oracle's, class agreement); the last two on
rank 0 at N = 1 only.
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


# Per-stage bound, as the rocprofv3 counters of profiles/ show it: VALU = VALU-issue-bound (>= 1/2 of
# the SIMD's VALU issue busy), latency = memory-latency-bound (SQ wait > 0.6 of wave cycles at full occupancy).
STAGE_BOUND = {"anchor_test": "valu", "requery": "latency+valu", "spill_search": "latency", "nvt1": "valu",
               "nvt2": "valu", "flat_phase": "latency", "edge_phase": "latency", "corner_phase": "latency",
               "finish": "-"}


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
        return [f"k_knn_anchor<{c}, {2 * c}>", f"k_knn_requery<{2 * c}, false, 64>", f"k_knn_redo_wave<{2 * c}, false>",
                f"k_nvt1<{c}, {unit}>"]
    return [f"k_knn_nvt1<{c}, {'true' if seeding else 'false'}>"]


def b_alg_iteration(k, ku):
    """Algorithmic bytes / point / iteration: 148 + 72k + 60k_u."""
    return 148 + 72 * k + 60 * ku


def b_alg_knn_nvt1(k):
    """Fused kNN + NVT1 kernel: query xyz 12 + k winners' snapshot xyz 12k + list write 4k (kNN) + current
    v_j, n_j 24k + own n 12 + f_n write 12 (NVT1, the list and own position come from registers)."""
    return 12 + 12 * k + 4 * k + 24 * k + 12 + 12


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
    b = float(tj["per_iteration_bytes"])
    return {"bytes_per_iteration": b, "achieved": round(b / (ms_per_step / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(b / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "source": tj.get("source", "profiles/traffic.json")}


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
    ap.add_argument("--no-rebalance", dest="rebalance", action="store_false",
                    help="slab mode: keep the equal-count cut (default: re-cut by class cost after warm-up 2)")
    ap.add_argument("--no-ten", dest="ten", action="store_false",
                    help="skip the ten_iteration_ms measurement (fresh cloud, 10 iterations incl. the first)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # RCCL ("nccl") between GPUs; PCD_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU
        backend = os.environ.get("PCD_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    mode = "single" if world == 1 else ("replicas" if args.replicas else "slab")

    if mode == "slab":
        # one global cloud of world x P points (identical on every rank), cut into spatial slabs with a halo
        from pcd_slab import SlabDenoiser, TorchTransport
        total = args.points if args.strong else args.points * world
        # one cloud, sampled on rank 0 only and broadcast (device sampling is not bit-reproducible across ranks);
        # d = 2 l (Processor.py:120-121) likewise on rank 0 only: the other ranks never grid the whole cloud
        if rank == 0:
            pos, nrm, diag = make_cloud(total, 3, dev)
            dt = torch.tensor([2 * float(Processor(Pointcloud(pos), k_hint=args.k).meanEdgeLength())], device=dev)
        else:
            pos = torch.empty((total, 3), dtype=torch.float32, device=dev)
            nrm = torch.empty_like(pos)
            dt = torch.zeros(1, device=dev)
        dist.broadcast(pos, 0)
        dist.broadcast(nrm, 0)
        dist.broadcast(dt, 0)
        d = float(dt)
        # coverage checked every 10 iterations (a thin halo re-plans and replays, pcd_slab); slabs re-cut by class
        # cost after the second warm-up iteration (rebalance), so the timed region runs on the balanced plan
        sd = SlabDenoiser(pos, nrm, max(args.k, args.k_update), transport=TorchTransport(), k_hint=args.k,
                          seeding=args.seeding, check_every=10)
        del pos, nrm
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
        if mode == "slab" and args.rebalance and w == min(1, args.warmup - 2):
            sd.rebalance()         # cost-weighted cut from this iteration's classes (next iteration re-anchors)
    if mode != "slab":
        fused.set_timing(True)     # per-stage HIP events on the launch stream, every timed iteration
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
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ms_per_step = elapsed / args.steps * 1e3
    total_points = args.points if (mode == "slab" and args.strong) else args.points * world
    value = total_points / (ms_per_step / 1e3) / 1e6

    # per-kernel timing (HIP events on the launch stream), outside the timed region
    kernel_ms, knn_ms = {}, float("nan")
    if mode == "slab":
        sd.check()      # exactness: no k-ball left its rank's slab + halo
        ks = [sd.iterate_timed(params) for _ in range(args.profile_steps)]
        if ks:
            kernel_ms = {key: round(float(np.mean([x[key] for x in ks])), 4) for key in ks[0]}
            knn_ms = kernel_ms["knn_nvt1"]
    else:
        slots = fused.timing()      # averages over exactly the timed iterations
        fused.set_timing(False)
        fused.check()               # device error word: invalid list entries would fail the bench here
        if slots:
            names = nat.FusedDenoiser.TIMING_SLOTS
            kernel_ms = {names[i]: round(float(slots[i]), 4) for i in range(min(len(slots), len(names)))}
            knn_ms = float(sum(slots[:4]))
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

    k1_points = sd.owned_global.numel() if mode == "slab" else args.points
    k1_bytes = b_alg_knn_nvt1(args.k) * k1_points
    achieved = k1_bytes / (knn_ms / 1e3) / 1e9 if knn_ms == knn_ms else None
    k1_names = k1_kernels(args.k, args.k_update, args.seeding, args.anchoring)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile) and mode != "slab":
        try:
            tj = json.load(open(tfile))
            if tj.get("points") == args.points and tj.get("k") == args.k:
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
                                "a missing blob)") + ", k=32, k_u=8, 1 iteration per step",
                   "points_per_gpu": total_points // world, "k": args.k, "k_update": args.k_update,
                   "global_points": total_points,
                   "parallelism": {"single": "single", "replicas": f"replicas x{world}",
                                   "slab": f"spatial slabs x{world}"}[mode]},
        "iterations_per_sec": round(1e3 / ms_per_step, 2),
        "first_iteration_ms": round(first_ms, 3) if first_ms is not None else None,
        "ten_iteration_ms": round(ten_ms, 3) if ten_ms is not None else None,
        "chamfer": chamfer,
        "kernel_ms": kernel_ms,
        "stage_bound": STAGE_BOUND if mode != "slab" else None,
        "iteration_roofline": {"bound": "hbm", "alg_bytes_per_point": b_alg_iteration(args.k, args.k_update),
                               "achieved": round(iter_alg / (ms_per_step / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s",
                               "frac": round(iter_alg / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
        "measured_traffic": measured_traffic(args.points, args.k, ms_per_step) if mode != "slab" else None,
        "roofline": {"kernel": "K1 stage (kNN + NVT1): " + " + ".join(k1_names), "bound": "valu+latency",
                     "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "alg_bytes_per_launch": k1_bytes, "avg_launch_ms": round(knn_ms, 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["parity"] = cpu_baseline(args.k, args.k_update, args.cpu_sample, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
