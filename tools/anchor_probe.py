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
    # (K', lambda): anchor lists of K' points; a failing query is re-anchored at q + lambda * (q - q_prev)
    variants = [(64, 0.0), (64, -0.5), (64, -0.25), (64, -1.0)]
    idx0 = {}
    for kp in sorted({v[0] for v in variants}):
        idx0[kp] = grid.knn(snap, kp, with_d2=True)
    anchors = {v: [snap.clone(), idx0[v[0]][0].clone(), idx0[v[0]][1][:, -1].sqrt()] for v in variants}
    prev = snap.clone()
    cur = torch.empty_like(snap)
    for it in range(1, iters + 1):
        fused.iterate(params, 1)
        fused.store(cur)
        mv = (cur - prev).norm(dim=1)
        line = f"it {it}: moved>0 {float((mv > 0).float().mean()):.3f}"
        for (kp, lam), (a, S, D) in anchors.items():
            delta = (cur - a).norm(dim=1)
            fail = torch.zeros(n, dtype=torch.bool, device=dev)
            for c0 in range(0, n, 2_000_000):                     # chunks: [n, kp] distance blocks
                sl = slice(c0, min(n, c0 + 2_000_000))
                dS = (snap[S[sl]] - cur[sl, None, :]).norm(dim=2)
                kth = dS.kthvalue(k, dim=1).values
                fail[sl] = ~(kth < (D[sl] - delta[sl]) * (1 - 1e-5))
                del dS
            line += f" | K'={kp} lam={lam:g} fail {float(fail.float().mean()) * 100:5.2f}%"
            if fail.any():
                fi = fail.nonzero().squeeze(1)
                at = cur[fi] + lam * (cur[fi] - prev[fi])
                i2, dd2 = grid.knn(at, kp, with_d2=True)
                a[fi] = at
                S[fi] = i2
                D[fi] = dd2[:, -1].sqrt()
        print(line, flush=True)
        prev.copy_(cur)


if __name__ == "__main__":
    main()
