"""A/B timing of the anchored K1 (anchor test + NVT1) on a fixed state (diagnostic, not a test).
The snapshot positions are reloaded after one dense pass, so every query certifies and only k_knn_anchor_nvt1
runs; repeated K1 stages on that state are timed with HIP events.  usage: python tools/k1_probe.py [n ...]"""
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
    for n in [int(x) for x in (sys.argv[1:] or ["10000000"])]:
        pos, nrm, _ = make_cloud(n, 2, dev)
        proc = Processor(Pointcloud(pos, nrm), k_hint=32)
        d = 2 * float(proc.meanEdgeLength())
        params = nat.make_params(k=32, k_update=8, d=d)
        fused = nat.FusedDenoiser(proc.selector.grid, 32)
        fused.load(pos, nrm)
        fused.iterate(params, 1)          # dense anchoring at the snapshot
        fused.load(pos, nrm)
        fused.stage(params, nat.STAGE_KNN_NVT1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            fused.stage(params, nat.STAGE_KNN_NVT1)
        e1.record()
        torch.cuda.synchronize()
        print(f"n={n}: anchored K1 on the snapshot state {e0.elapsed_time(e1) / reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
