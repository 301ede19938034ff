"""K1 (kNN + NVT1) time with and without the seeded capped search, per cloud size (diagnostic, not a test)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in (sys.argv[1:] or ["1000000", "10000000"])]:
        pos, nrm, _ = make_cloud(n, 2, dev)
        proc = Processor(Pointcloud(pos, nrm), k_hint=32)
        d = 2 * float(proc.meanEdgeLength())
        params = nat.make_params(k=32, k_update=8, d=d)
        for seeding in (False, True):
            fused = nat.FusedDenoiser(proc.selector.grid, 32)
            fused.load(pos, nrm)
            fused.set_seeding(seeding)
            fused.iterate(params, 2)
            fused.set_timing(True)
            ts = []
            for _ in range(5):
                fused.iterate(params, 1)
                ts.append(sum(fused.timing()[:4]))
            print(f"n={n} seeding={seeding}: K1 {sum(ts)/len(ts):.3f} ms  {['%.2f' % t for t in ts]}", flush=True)
            del fused


if __name__ == "__main__":
    main()
