"""Time the dense first re-anchoring alone (diagnostic, not a test): one K1 stage of a fresh denoiser (every row
re-anchored by k_dense_radius + k_knn_dense_q<64, 2>) at 10M points, nothing after it -- safe for timing-experiment builds whose
lists are wrong (no later stage gathers through them).  usage: PCD_LIB=... python tools/dense_probe.py [n] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
import pcd_native as nat  # noqa: E402
from bench import make_cloud  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 2, dev)
    grid = nat.Grid(pos, k_hint=32)
    p = nat.make_params(k=32, k_update=8, d=0.01)
    ts = []
    for _ in range(reps):
        fd = nat.FusedDenoiser(grid, 32)
        fd.load(pos, nrm)
        fd.set_timing(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        fd.stage(p, nat.STAGE_KNN_NVT1)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
        st = fd.tile_stats()
        del fd
    print(f"dense K1 stage at {n:,} points: {' '.join(f'{t:.2f}' for t in ts)} ms  (spilled {st['spilled']}, big box {st['spilled_big_box']}, ambiguous {st['spilled_ambiguous']})", flush=True)


if __name__ == "__main__":
    main()
