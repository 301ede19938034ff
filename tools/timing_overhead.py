"""Cost of the per-stage HIP events inside the timed region (diagnostic, not a test): the bench cloud at 10M points,
iterations 6-25 of the same cloud (reloaded, anchors reset) timed with stage timing off / on, three trials each,
alternating; ms per iteration by the host clock around the 20 iterations.  usage: python tools/timing_overhead.py [points]"""
import os
import sys
import time

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
    dev = torch.device("cuda", 0)
    pos, nrm, _diag, _surf = make_cloud(n, 2, dev, clean=True)
    proc = Processor(Pointcloud(pos, nrm), k_hint=32)
    d = 2 * float(proc.meanEdgeLength())
    fused = proc._fused_for(32)
    params = nat.make_params(k=32, k_update=8, d=d)
    res = {False: [], True: []}
    for trial in range(6):
        on = trial % 2 == 1
        # the same cloud from scratch each trial: iterations 1-5 untimed, 6-25 timed (the bench's window)
        fused.load(proc.graph.pos, proc.graph.n)
        fused.reset_seed()
        fused.iterate(params, 5)
        fused.set_timing(on)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fused.iterate(params, 1)
        torch.cuda.synchronize()
        res[on].append((time.perf_counter() - t0) / 20 * 1e3)
        if on:
            fused.timing()
    fused.set_timing(False)
    for on in (False, True):
        print(f"stage timing {'on ' if on else 'off'}: " + " ".join(f"{x:.4f}" for x in res[on]) + " ms/iteration",
              flush=True)


if __name__ == "__main__":
    main()
