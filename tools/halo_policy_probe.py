"""Which band / sphere policy keeps the slabs exact through a run (diagnostic, not a test)?  configs[4]'s 80M-point
cloud, the equal-count cut into `world` slabs, the single-GPU fused loop for `iters` iterations; for every row within
4e-3 of a face it records, before each iteration, the exact reach of its k-ball past its slab's faces at its CURRENT
position, d_k there and its displacement from the snapshot.  Then, for a plan made after iteration t (the state a
re-plan gathers) covering the next h iterations, it prices each policy -- band = margin x q999 of the predicted need,
spheres for the rows above it -- by the rows the run would have failed and the halo rows per rank (SlabPlan.build).
Prediction: need = reach_t + g * j * (s_r + s_f) for the j-th iteration ahead, s_r = the row's own mean speed so
far (D_t / t), s_f = a speed floor (a quantile of s_r).  usage: python tools/halo_policy_probe.py [points] [world] [iters]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402
from pcd_slab import SlabPlan, Spheres, _cut  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402


def q(x, p):
    return float(torch.sort(x).values[int(p * (x.numel() - 1))]) if x.numel() else 0.0


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 80_000_000
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 3, dev)
    d = 2 * float(Processor(Pointcloud(pos), k_hint=32).meanEdgeLength())
    axis, key, owner, lo, hi = _cut(pos, world)
    lo_a = torch.tensor(lo, device=dev)[owner]
    hi_a = torch.tensor(hi, device=dev)[owner]
    first, last = owner == 0, owner == world - 1
    gap = torch.minimum(torch.where(last, torch.full_like(key, 1e9), hi_a - key),
                       torch.where(first, torch.full_like(key, 1e9), key - lo_a))
    idx = torch.nonzero(gap < 4e-3).flatten()
    lo_t, hi_t, fi, la = lo_a[idx], hi_a[idx], first[idx], last[idx]
    del lo_a, hi_a, gap
    m = idx.numel()
    print(f"{n:,} points, {world} slabs, d {d:.4g}, {m:,} rows within 4e-3 of a face", flush=True)
    R = torch.empty((iters + 1, m), device=dev)      # reach before iteration t (t = 1..iters), row 0 unused
    K = torch.empty((iters + 1, m), device=dev)      # d_k there
    D = torch.empty((iters + 1, m), device=dev)      # displacement from the snapshot there
    g = nat.Grid(pos, k_hint=nat.fused_k_hint(32) or 32)
    fd = nat.FusedDenoiser(g, 32)
    fd.load(pos, nrm)
    params = nat.make_params(k=32, k_update=8, d=d)
    cur = pos.clone()
    for t in range(1, iters + 1):
        qp = cur[idx].contiguous()
        _, d2 = g.knn(qp, 32, with_d2=True, idx_bits=32)
        dk = d2[:, -1].sqrt()
        del d2
        kq = qp[:, axis]
        up = torch.where(la, torch.full_like(dk, -1e9), kq + dk - hi_t)
        down = torch.where(fi, torch.full_like(dk, -1e9), lo_t - kq + dk)
        R[t], K[t], D[t] = torch.maximum(up, down), dk, (qp - pos[idx]).norm(dim=1)
        fd.iterate(params, 1)
        fd.store(cur)
    del fd
    torch.cuda.empty_cache()
    own = torch.bincount(owner, minlength=world)

    def evaluate(tag, t, h, band, sph, rad):
        """t: the plan's state is before iteration t+1 (after t iterations); it covers iterations t+1 .. t+h."""
        span = range(t + 1, min(t + h, iters) + 1)
        bad_band = sum(int(((R[j] > band) & ~sph).sum()) for j in span)
        ratio = max((float(((D[j] + K[j])[sph] / rad[sph]).max()) if bool(sph.any()) else 0.0) for j in span)
        sid = idx[sph]
        sp = Spheres.around(pos, sid, rad[sph] * 1.0, owner) if sid.numel() else None
        plan = SlabPlan.build(pos, world, band, spheres=sp)
        halo = max(int(plan.local[r].numel() - own[r]) for r in range(world))
        print(f"  {tag}: band {band:.4g} ({band / d:.2f} d), spheres {int(sph.sum()):,}, failing band rows {bad_band:,}, "
              f"sphere ratio max {ratio:.3f}, halo rows/rank {halo:,}", flush=True)

    # how the need grows after iteration 1, by the row's displacement in iteration 1 (s1, units of d)
    s1 = D[2] / d
    bins = [(0.0, 0.05), (0.05, 0.1), (0.1, 0.25), (0.25, 0.5), (0.5, 0.75), (0.75, 1.01)]
    for lo_, hi_ in bins:
        m_ = (s1 >= lo_) & (s1 < hi_) & (R[2] > -1e8)
        if not bool(m_.any()):
            continue
        row = []
        for j in range(4, iters + 1, 3):
            gr = (R[j] - R[2])[m_] / d
            gs = (D[j] + K[j] - K[2])[m_] / d
            row.append(f"j{j}: reach +{q(gr, 0.999):.2f}/{float(gr.max()):.2f} ball {q(gs, 0.999):.2f}/{float(gs.max()):.2f}")
        print(f"s1 in [{lo_}, {hi_}) d ({int(m_.sum()):,} rows): " + "; ".join(row), flush=True)
    # cut_spheres' policy: need = reach + d (lead + 0.8 sqrt(ahead) + 0.2 ahead), spheres of 1.1 (D + d_k + d (lead + 2.4 sqrt(ahead)))
    for t, h in ((0, 1), (0, 2), (1, 7), (1, iters - 1)):
        print(f"plan after iteration {t}, covering iterations {t + 1}..{t + h}:", flush=True)
        ahead = h - 1
        lead = 1.75 if (t == 0 and ahead > 0) else 0.0
        need = (R[t + 1] + d * (lead + 0.8 * ahead ** 0.5 + 0.2 * ahead)).clamp(min=0)
        valid = R[t + 1] > -1e8
        band = 1.25 * max(q(need[valid], 0.999), q(K[t + 1][valid], 0.5))
        sph = (1.25 * need > band) & valid
        rad = torch.maximum(1.5 * K[t + 1], 1.1 * (D[t + 1] + K[t + 1] + d * (lead + 2.4 * ahead ** 0.5)))
        evaluate("cut_spheres", t, h, band, sph, rad)

if __name__ == "__main__":
    main()
