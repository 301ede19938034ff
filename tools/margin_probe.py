"""Diagnostics (not a test): anchored-kNN failure rate as a function of the anchor radius.

An anchor (a, D) certifies the k-NN of the current position q when d_k(q) + |q - a| < D (every snapshot point
outside ball(a, D) is in the anchor's list).  The list a radius-D anchor must hold is |ball(a, D)|.  For each
variant the probe keeps one simulated anchor per point, re-anchors the failing points at q, and prints the failure
rate per iteration and the mean list size of the re-anchored points.
  KA=64   : D = the 64th neighbour distance at a (the shipped scheme)
  beta=b  : D = b * d_k(a)                       (radius anchors; list size = count within D)
usage: python tools/margin_probe.py [n_points] [iterations]
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 25
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

    def dk_of(x, kk=k):
        out = torch.empty(x.size(0), device=dev)
        for c0 in range(0, x.size(0), 2_000_000):
            _, d2 = grid.knn(x[c0:c0 + 2_000_000], kk, with_d2=True, idx_bits=32)
            out[c0:c0 + 2_000_000] = d2[:, -1].sqrt()
        return out

    def count_within(x, r):
        c = torch.empty(x.size(0), dtype=torch.int64, device=dev)
        L = nat.lib()
        for c0 in range(0, x.size(0), 1_000_000):
            xs, rs = x[c0:c0 + 1_000_000].contiguous(), r[c0:c0 + 1_000_000].contiguous()
            cs = torch.empty(xs.size(0), dtype=torch.int64, device=dev)
            nat.check(L.pcd_radius_count(grid.handle, nat.ptr(xs), xs.size(0), nat.ptr(rs), nat.ptr(cs),
                                         nat.c_void_p(nat.stream_ptr())), "radius_count")
            c[c0:c0 + xs.size(0)] = cs
        return c

    d64 = dk_of(snap, 64)
    d32 = dk_of(snap, 32)
    betas = [1.4, 1.6, 1.8, 2.0]
    anchors = {"KA=64": [snap.clone(), d64.clone()]}
    for b in betas:
        anchors[f"beta={b}"] = [snap.clone(), b * d32]
    sizes = {name: [] for name in anchors}
    for name, (a, D) in anchors.items():
        smp = torch.randperm(n, device=dev)[:200_000]
        sizes[name].append(float(count_within(a[smp], D[smp]).float().mean()))
    print(f"n={n} d=2l={d:.4g} median d32={float(d32.median()):.4g} d={d / float(d32.median()):.3f} d32", flush=True)
    print("initial list sizes: " + " ".join(f"{k_}:{v[0]:.0f}" for k_, v in sizes.items()), flush=True)
    prev = snap.clone()
    cur = torch.empty_like(snap)
    for it in range(1, iters + 1):
        fused.iterate(params, 1)
        fused.store(cur)
        mv = (cur - prev).norm(dim=1)
        dkq = dk_of(cur)
        rel = mv / dkq
        line = (f"it {it:2d}: step/d_k p50 {float(rel.median()):.3f} p90 {float(rel.quantile(0.9)) if n <= 16_000_000 else 0:.3f}"
                f" moving>0.25d_k {float((rel > 0.25).float().mean()) * 100:5.2f}%")
        for name, (a, D) in anchors.items():
            fail = ~((dkq + (cur - a).norm(dim=1)) < D * (1 - 1e-5))
            line += f" | {name} {float(fail.float().mean()) * 100:5.2f}%"
            fi = fail.nonzero().squeeze(1)
            if fi.numel():
                a[fi] = cur[fi]
                if name == "KA=64":
                    D[fi] = dk_of(cur[fi], 64)
                else:
                    D[fi] = float(name.split("=")[1]) * dkq[fi]
                    if it in (5, 20):
                        sm = fi[torch.randperm(fi.numel(), device=dev)[:100_000]]
                        sizes[name].append(float(count_within(cur[sm], D[sm]).float().mean()))
        print(line, flush=True)
        prev.copy_(cur)
    print("list sizes (initial, it5, it20 re-anchors): " +
          " ".join(f"{k_}:{'/'.join(f'{x:.0f}' for x in v)}" for k_, v in sizes.items()), flush=True)


if __name__ == "__main__":
    main()
