"""Diagnostics for the kNN grid on the GPU: grid stats and timings vs cell size / k (not a test)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = torch.device("cuda", 0)
    pos, nrm, diag = make_cloud(n, 2, dev)
    g0 = nat.Grid(pos, k_hint=32)
    info = g0.info()
    print("auto grid:", info, "pts/cell", n / info["cells"])
    perm = g0.perm().long()
    qs = pos[perm].contiguous()   # queries in Morton order (like the fused loop)
    for scale in (0.5, 0.7, 1.0, 1.4, 2.0):
        g = nat.Grid(pos, k_hint=32, cell=info["cell"] * scale)
        inf = g.info()
        for k in (8, 32):
            ms = timeit(lambda: g.knn(qs, k))
            print(f"cell x{scale}: cells={inf['cells']} pts/cell={n/inf['cells']:.1f} k={k}: {ms:.3f} ms "
                  f"({n/ms/1e3:.1f} Mq/s) {g.knn_stats(qs, k)}")
    ms = timeit(lambda: g0.knn(pos, 32))
    print(f"auto grid, queries in ORIGINAL (random) order, k=32: {ms:.3f} ms")


if __name__ == "__main__":
    main()
