"""Halo rows of the slab plans of configs[4]'s 80M-point cloud (diagnostic, not a test): the coverage-sphere plan
(cut_spheres) at its first band and after one thin-halo re-plan (band x2), with the spheres scaled alike or kept,
for two sphere margins -- geometry only, no iterations.  usage: python tools/halo_plan_probe.py [points] [world]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
from bench import make_cloud  # noqa: E402
from pcd_slab import SlabPlan, Spheres, _cut, cut_spheres  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 80_000_000
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    pos, _, _ = make_cloud(n, 3, dev)
    for sm in (1.25, 1.5):
        band, ids, rad = cut_spheres(pos, world, 32, sphere_margin=sm)
        for bscale, sscale in ((1.0, 1.0), (2.0, 2.0), (2.0, 1.0)):
            sp = Spheres.around(pos, ids, rad * sscale, _cut(pos, world)[2])
            plan = SlabPlan.build(pos, world, band * bscale, spheres=sp)
            own = torch.bincount(plan.owner, minlength=world)
            halo = [int(plan.local[r].numel() - own[r]) for r in range(world)]
            print(f"sphere margin {sm}: {ids.numel():,} spheres, band {band * bscale:.3g} (x{bscale}), spheres x{sscale}:"
                  f" halo rows {halo} (max {max(halo):,})", flush=True)


if __name__ == "__main__":
    main()
