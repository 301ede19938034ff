"""How far do the k-balls of the points near a slab face drift from the snapshot (diagnostic, not a test)?  configs[4]'s
80M-point cloud, the equal-count cut into `world` slabs with cut_spheres' band + spheres, the single-GPU fused loop:
before each iteration t, the exact reach past the owning slab's faces of every near-face row's k-ball at its CURRENT
position (Grid.knn against the snapshot, as K1 searches), the band the sphere-less rows need, the spheres' worst
ratio, and the displacement from the snapshot (near rows / all rows) against t x d (every step is clamped below d,
Denoiser.py's `norm < d` keeps).  usage: python tools/halo_drift_probe.py [points] [world] [iterations]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402
from pcd_slab import SlabPlan, Spheres, _cut, _cut_reach, cut_spheres  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 80_000_000
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 3, dev)
    d = 2 * float(Processor(Pointcloud(pos), k_hint=32).meanEdgeLength())
    band, sid, srad = cut_spheres(pos, world, 32)
    plan = SlabPlan.build(pos, world, band, spheres=Spheres.around(pos, sid, srad, _cut(pos, world)[2]))
    own = torch.bincount(plan.owner, minlength=world)
    halo_rows = max(int(plan.local[r].numel() - own[r]) for r in range(world))
    idx, reach0, dk0, _ = _cut_reach(pos, world, 32)
    axis, key, owner, lo, hi = _cut(pos, world)
    lo_t = torch.tensor(lo, device=dev)[owner[idx]]
    hi_t = torch.tensor(hi, device=dev)[owner[idx]]
    first, last = owner[idx] == 0, owner[idx] == world - 1
    sph = torch.isin(idx, sid.to(dev))
    R = torch.zeros(n, device=dev)
    R[sid.to(dev)] = srad.to(dev)
    R = R[idx]
    print(f"{n:,} points, {world} slabs: d {d:.4g}, band {band:.4g}, {sid.numel():,} spheres, near rows "
          f"{idx.numel():,}, halo rows/rank (max) {halo_rows:,}", flush=True)
    g = nat.Grid(pos, k_hint=nat.fused_k_hint(32) or 32)
    fd = nat.FusedDenoiser(g, 32)
    fd.load(pos, nrm)
    params = nat.make_params(k=32, k_update=8, d=d)
    cur = pos.clone()
    for t in range(1, iters + 1):
        q = cur[idx].contiguous()
        _, d2 = g.knn(q, 32, with_d2=True, idx_bits=32)
        dk = d2[:, -1].sqrt()
        kq = q[:, axis]
        up = torch.where(last, torch.zeros_like(dk), kq + dk - hi_t)
        down = torch.where(first, torch.zeros_like(dk), lo_t - kq + dk)
        reach = torch.maximum(up, down)
        need = float(reach[~sph].max()) if bool((~sph).any()) else 0.0
        disp = (cur - pos).norm(dim=1)
        ratio = float(((disp[idx] + dk)[sph] / R[sph]).max()) if bool(sph.any()) else 0.0
        grow = float((reach - reach0)[~sph].max())
        print(f"iteration {t}: band needed {need:.4g} ({need / band:.3f} x band), reach growth max {grow:.4g} "
              f"({grow / d:.2f} d), sphere ratio max {ratio:.3f}, displacement near {float(disp[idx].max()):.4g} "
              f"({float(disp[idx].max()) / d:.2f} d) all {float(disp.max()):.4g} ({float(disp.max()) / d:.2f} d), "
              f"p99.9 near {float(torch.sort(disp[idx]).values[int(0.999 * (idx.numel() - 1))]):.3g}", flush=True)
        del d2
        fd.iterate(params, 1)
        fd.store(cur)


if __name__ == "__main__":
    main()
