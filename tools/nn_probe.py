"""Public nearest-neighbour path at full size (diagnostic): grid build and k = 1 queries of TorchUtils.ChamferDistance
on the bench workload, timed separately.  usage: python tools/nn_probe.py [n]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    pos, nrm, _, surf = make_cloud(n, 2, dev, clean=True)
    for k_hint in (1, 8, 32):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = nat.Grid(surf, k_hint=k_hint)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        idx, d2 = g.knn(pos, 1, with_d2=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"k_hint {k_hint}: grid {1e3 * (t1 - t0):.1f} ms  knn(k=1) {1e3 * (t2 - t1):.1f} ms  "
              f"mean d2 {float(d2.mean()):.3e}", flush=True)


if __name__ == "__main__":
    main()
