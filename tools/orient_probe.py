"""Time GraphBuilder.flipNormals' device MST orientation against the host Kruskal + DFS on a synthetic surface.

    python tools/orient_probe.py --n 1000000 10000000 --k 12
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"), ROOT]
import pcd_native as nat  # noqa: E402
from Pointcloud.Modules.GraphBuilder import GraphBuilder  # noqa: E402
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402


def surface(m, seed=0):
    g = torch.Generator().manual_seed(seed)
    uv = torch.rand(m, 2, generator=g) * 4 - 2
    z = torch.sin(uv[:, 0] * 2) * torch.cos(uv[:, 1] * 3) * 0.4
    return torch.cat([uv, z[:, None]], 1) + 0.001 * torch.randn(m, 3, generator=g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1_000_000, 10_000_000])
    ap.add_argument("--k", type=int, default=12)
    ap.add_argument("--host-max", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = nat.device()
    for m in args.n:
        pos = surface(m).to(dev)
        gb = GraphBuilder(Pointcloud(pos))
        ei = gb.getKNNEdgeIndex(args.k)
        n = gb.getPVTDecompositionWithKNN(ei)[..., 0].contiguous()
        a, b = ei[0].contiguous(), ei[1].contiguous()
        out = nat.orient_normals_mst_gpu(pos, n, a, b)          # warm-up (allocations, code objects)
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            out = nat.orient_normals_mst_gpu(pos, n, a, b)
        torch.cuda.synchronize()
        gpu_ms = (time.perf_counter() - t0) / reps * 1e3
        rec = {"points": m, "edges": a.numel(), "gpu_ms": round(gpu_ms, 2)}
        if m <= args.host_max:
            hp, hn, ha, hb = pos.cpu(), n.cpu().clone(), a.cpu(), b.cpu()
            t0 = time.perf_counter()
            nat.orient_normals_mst(hp, hn, ha, hb)
            rec["host_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
            rec["bitwise_equal"] = bool(torch.equal(hn, out.cpu()))
        print(json.dumps(rec), flush=True)
        del pos, gb, ei, n, a, b, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
