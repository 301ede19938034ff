"""How wide are the anchor sets in snapshot-rank (Morton) order?  Sizing study for the compact anchor sets tried in
round 5 (four bases + 16-bit codes a row; measured and reverted, DESIGN.md §3 "tried"): the 64 nearest of a point, sorted by rank, cut greedily into clusters of span < 2^b;
prints the fraction of rows that need more than 1..4 clusters.  CPU only (scipy), a noisy torus surface.

    python tools/aset_span.py [--points 2000000]

Measured (2M points, every 20th row): one 16-bit window misses 9.1 % of the sets; four 14-bit windows miss none of
the 10^5 sampled rows (three miss 0.17 %).
"""
import argparse

import numpy as np
import scipy.spatial as sp


def spread(x):
    x = x.astype(np.uint64) & np.uint64(0x1FFFFF)
    for s, m in [(32, 0x1F00000000FFFF), (16, 0x1F0000FF0000FF), (8, 0x100F00F00F00F00F), (4, 0x10C30C30C30C30C3),
                 (2, 0x1249249249249249)]:
        x = (x | (x << np.uint64(s))) & np.uint64(m)
    return x


def clusters(s, w):
    n = np.ones(len(s), int)
    start = s[:, 0].copy()
    for t in range(1, s.shape[1]):
        new = s[:, t] >= start + w
        n += new
        start = np.where(new, s[:, t], start)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=2_000_000)
    ap.add_argument("--ka", type=int, default=64)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    n = a.points
    u, v = rng.random(n) * 2 * np.pi, rng.random(n) * 2 * np.pi
    R, r = 1.0, 0.35
    p = np.stack([(R + r * np.cos(v)) * np.cos(u), (R + r * np.cos(v)) * np.sin(u), r * np.sin(v)], 1)
    p = (p + rng.normal(0, 0.003, p.shape)).astype(np.float32)
    h = np.sqrt(16 * 4 * np.pi ** 2 * R * r / n)            # ~16 points a surface cell, as the grid sizes them
    c = ((p - p.min(0)) / h).astype(np.int64)
    key = spread(c[:, 0]) | (spread(c[:, 1]) << np.uint64(1)) | (spread(c[:, 2]) << np.uint64(2))
    p = p[np.argsort(key, kind="stable")]
    _, ix = sp.cKDTree(p).query(p[::20], k=a.ka, workers=8)
    s = np.sort(ix, 1)
    for bits in (16, 15, 14, 13):
        nc = clusters(s, 1 << bits)
        print(f"{bits}-bit windows: rows needing more than 1/2/3/4 =",
              " ".join(f"{(nc > m).mean():.5f}" for m in (1, 2, 3, 4)))


if __name__ == "__main__":
    main()
