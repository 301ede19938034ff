"""Anchored kNN over a long run (diagnostic, not a test): per iteration, the rows that failed the anchor test and
the HIP-event time of K1 / the whole iteration.  usage: python tools/redo_probe.py [n] [iterations]"""
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
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 2, dev)
    proc = Processor(Pointcloud(pos, nrm), k_hint=32)
    d = 2 * float(proc.meanEdgeLength())
    params = nat.make_params(k=32, k_update=8, d=d)
    fused = proc._fused_for(32)
    fused.load(proc.graph.pos, proc.graph.n)
    fused.set_timing(True)
    for it in range(1, iters + 1):
        fused.iterate(params, 1)
        t = fused.timing()
        r = fused.redo_rows()
        extra = ""
        if hasattr(fused, "tile_stats"):
            ts = fused.tile_stats()
            extra += (f"  | spilled to the exact wave search {ts['spilled']} (big box {ts['spilled_big_box']}, "
                      f"ambiguous {ts['spilled_ambiguous']})")
        print(f"it {it:3d}: redo {r:9d} ({r / n * 100:5.2f} %)  K1 {sum(t[:4]):7.3f} ms (requery {t[1]:6.3f})  iteration {sum(t):7.3f} ms{extra}",
              flush=True)


if __name__ == "__main__":
    main()
