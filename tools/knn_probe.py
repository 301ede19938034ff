"""Diagnostics for the kNN grid on the GPU (not a test): the insertion and batched searches side by side, per cell
size and k, with their work counters.  usage: python tools/knn_probe.py [n_points]"""
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
    print("auto grid:", info, "pts/cell", round(n / info["cells"], 2), flush=True)
    perm = g0.perm().long()
    qs = pos[perm].contiguous()   # queries in Morton order (like the fused loop)
    for scale in (0.7, 1.0, 1.4):
        g = nat.Grid(pos, k_hint=32, cell=info["cell"] * scale)
        inf = g.info()
        for k in (16, 32):
            ms = timeit(lambda: g.knn(qs, k))
            line = f"cell x{scale} pts/cell={n/inf['cells']:.1f} k={k}: production {ms:.3f} ms"
            for variant, name in ((0, "insertion"), (1, "batched")):
                ms_v = timeit(lambda: g.knn_stats(qs, k, batched=bool(variant)), reps=3)
                line += f" | {name} {ms_v:.3f} ms {g.knn_stats(qs, k, batched=bool(variant))}"
            print(line, flush=True)
    ms = timeit(lambda: g0.knn(pos, 32))
    print(f"auto grid, queries in ORIGINAL (random) order, k=32: {ms:.3f} ms")


if __name__ == "__main__":
    main()
