"""Diagnostics (not a test): how far do points move per denoise iteration relative to their k-th neighbour
distance, and how often would an "anchored" kNN list certify itself?

Anchor scheme: for query i keep (a_i, S_i, D_i) = an earlier position, the exact K'-NN of the snapshot at a_i and
the K'-th distance there.  At the current position q, delta = |q - a|; every snapshot point outside S_i is at least
D_i - delta away, so if the k-th distance of q over S_i is below D_i - delta, the k-NN of q is the top-k of S_i.
usage: python tools/anchor_probe.py [n_points] [iterations]
"""
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


def q(x, ps=(0.5, 0.9, 0.99, 0.999)):
    x = x.float()
    if x.numel() > 4_000_000:
        x = x[torch.randperm(x.numel(), device=x.device)[:4_000_000]]
    return " ".join(f"p{int(p*1000)/10:g}={torch.quantile(x, p).item():.3g}" for p in ps)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    k = 32
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 2, dev)
    snap = pos.clone()
    proc = Processor(Pointcloud(pos, nrm), k_hint=k)
    d = 2 * float(proc.meanEdgeLength())
    fused = proc._fused_for(k)
    fused.load(proc.graph.pos, proc.graph.n)
    params = nat.make_params(k=k, k_update=8, d=d)
    grid = proc.selector.grid
    print(f"n={n} d=2l={d:.4g}", flush=True)
    anchors = {}
    for kp in (40, 48, 64):
        idx, d2 = grid.knn(snap, kp, with_d2=True)
        anchors[kp] = [snap.clone(), idx, d2[:, -1].sqrt()]
    prev = snap.clone()
    cur = torch.empty_like(snap)
    for it in range(1, iters + 1):
        fused.iterate(params, 1)
        fused.store(cur)
        _, d2k = grid.knn(prev, k, with_d2=True)     # d_k at the position this iteration's kNN used
        dk = d2k[:, -1].sqrt()
        mv = (cur - prev).norm(dim=1)
        line = f"it {it}: move/d_k {q(mv / dk)}  moved>0 {float((mv > 0).float().mean()):.3f}"
        # certification at the NEXT query position (cur)
        for kp, (a, S, D) in anchors.items():
            delta = (cur - a).norm(dim=1)
            dS = (snap[S] - cur[:, None, :]).norm(dim=2)          # [n, kp]
            kth = dS.kthvalue(k, dim=1).values
            ok = kth < (D - delta) * (1 - 1e-5)
            fail = ~ok
            line += f" | K'={kp} fail {float(fail.float().mean()):.4f}"
            if fail.any():
                fi = fail.nonzero().squeeze(1)
                i2, dd2 = grid.knn(cur[fi], kp, with_d2=True)
                a[fi] = cur[fi]
                S[fi] = i2
                D[fi] = dd2[:, -1].sqrt()
            del dS
        print(line, flush=True)
        prev.copy_(cur)


if __name__ == "__main__":
    main()
