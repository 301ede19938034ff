"""CPSD driver time against the fused snapshot index's cell size (GPU box): pcd_cpsd_iterate on a denoiser built for
list caps 8 / 16 / 32 (about 8 / 16 / 32 points a cell), 1M and 50k bunny-sampled points, 50 iterations."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402

dev = torch.device("cuda", 0)
for n in (50_000, 1_000_000):
    pos, nrm, _ = make_cloud(n, 4, dev)
    d = 2 * float(Processor(Pointcloud(pos.clone(), nrm.clone()), k_hint=16).meanEdgeLength())
    for kmax in (8, 16, 32):
        proc = Processor(Pointcloud(pos.clone(), nrm.clone()), k_hint=16)
        dn = proc._fused_for(kmax)
        prm = nat.make_cpsd_params(r=d, d=d)
        dn.load(proc.graph.pos, proc.graph.n)
        dn.cpsd_iterate(prm, 2)
        dn.load(proc.graph.pos, proc.graph.n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dn.cpsd_iterate(prm, 50)
        torch.cuda.synchronize()
        print(f"n={n} kmax={kmax}: {(time.perf_counter() - t0) / 50 * 1e3:.4f} ms/iteration", flush=True)
