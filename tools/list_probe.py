"""Debug probe: per iteration, compare the fused loop's stored kNN lists (seeded / anchored) with the public grid
kNN of the same positions (exact, (d², index) order).  usage: python tools/list_probe.py [k] [iters] [fixture|N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd")]
import pcd_native as nat  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    src = sys.argv[3] if len(sys.argv) > 3 else "fandisk_k32"
    dev = nat.device()
    if src.isdigit():
        import bench
        pos, nrm, _ = bench.make_cloud(int(src), 2, dev)
        d = 2 * 0.8 * float(torch.sqrt(torch.tensor(0.0)) + 1e-3)
    else:
        f = np.load(os.path.join(ROOT, "tests", "golden", src + ".npz"))
        pos = torch.from_numpy(f["pos0"]).to(dev)
        nrm = torch.from_numpy(f["n0"]).to(dev)
        d = float(f["d"])
    g = nat.Grid(pos, k_hint=k)
    fd = nat.FusedDenoiser(g, max(k, 8))
    fd.load(pos, nrm)
    params = nat.make_params(k=k, k_update=8, d=d)
    kst = max(k, 8)
    p = torch.empty_like(pos)
    n = torch.empty_like(nrm)
    for it in range(iters):
        fd.store(p, n)                       # positions the next K1 queries
        fd.iterate(params, 1)
        got = fd.lists(kst)
        ref = g.knn(p, kst).to(torch.int64)
        bad = (got != ref).any(1)
        print(f"it {it + 1}: rows with a wrong list {int(bad.sum())} / {len(bad)}  redo {fd.redo_rows()}"
              f"  stats {fd.tile_stats()}")
        if bad.any():
            r = int(bad.nonzero()[0])
            print("  row", r, "got", got[r].tolist(), "\n  ref", ref[r].tolist())


if __name__ == "__main__":
    main()
