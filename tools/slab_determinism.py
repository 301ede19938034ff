"""Is the slab loop deterministic?  The same cloud through the same slab run twice (4 ranks sharing GPU 0 over the host
transport, cost-weighted re-cut after iteration 2), final owned states compared bit for bit -- a coverage re-plan
replays its iterations from a checkpoint and assumes the replay retraces them.  usage: python tools/slab_determinism.py [n]"""
import os
import socket
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd")]


def worker(rank, world, port, n, out, mode):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pcd_native as nat
    from bench import make_cloud
    from pcd_slab import SlabDenoiser, TorchTransport, gather_global
    dev = torch.device("cuda", 0)
    tr = TorchTransport()
    params = nat.make_params(k=32, k_update=8, d=0.0015)
    for run in range(2):
        pos = nrm = None
        if rank == 0:
            pos, nrm, _ = make_cloud(n, 3, dev)
            print(f"run {run}: cloud checksum {float(pos.double().sum()):.17g} {float((pos.double() ** 2).sum()):.17g}",
                  flush=True)
        if mode == "fresh" and run == 1:
            tr = TorchTransport()
        sd = SlabDenoiser(pos, nrm, 32, transport=tr, check_every=0, halo=0.01)
        sd.iterate(params, 2)
        if mode == "replan" and run == 1:
            sd._replan(sd.halo if rank == 0 else None)        # the same plan again: a new engine, same routes
        else:
            sd.rebalance()
        sd.iterate(params, 4)
        p, nn = gather_global(sd.owned_state(), sd.n_total, tr)
        st = sd.e.status()
        if rank == 0:
            np.savez(f"{out}_{run}.npz", pos=p.numpy(), n=nn.numpy(), status=st)
        del sd
        if mode == "fresh":
            tr.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    mode = sys.argv[2] if len(sys.argv) > 2 else "fresh"   # fresh: a new transport per run; shared; replan
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = os.path.join(ROOT, "gpurun_out", "slab_det")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    mp.spawn(worker, args=(4, port, n, out, mode), nprocs=4, join=True)
    a, b = np.load(f"{out}_0.npz"), np.load(f"{out}_1.npz")
    # the single-GPU fused loop on the same cloud and parameters
    import pcd_native as nat
    from bench import make_cloud
    dev = torch.device("cuda", 0)
    pos, nrm, _ = make_cloud(n, 3, dev)
    print(f"one GPU: cloud checksum {float(pos.double().sum()):.17g} {float((pos.double() ** 2).sum()):.17g}", flush=True)
    g = nat.Grid(pos, k_hint=nat.fused_k_hint(32) or 32)
    fd = nat.FusedDenoiser(g, 32)
    fd.load(pos, nrm)
    fd.iterate(nat.make_params(k=32, k_update=8, d=0.0015), 6)
    p1 = torch.empty_like(pos)
    fd.store(p1)
    p1 = p1.cpu().numpy()
    bbox = float(np.linalg.norm(p1.max(0) - p1.min(0)))
    for tag, x in (("run0", a), ("run1", b)):
        dp = np.linalg.norm(x["pos"] - p1, axis=1) / bbox
        print(f"{tag} vs one GPU: rows differing {np.mean(dp > 0):.6f}, p99 {np.percentile(dp, 99):.3g}, max {dp.max():.3g}",
              flush=True)
    dp = np.abs(a["pos"] - b["pos"]).max(1)
    print(f"[{mode}] slab determinism ({n} points, 4 ranks, 6 iterations, re-cut after 2): rows differing {np.mean(dp > 0):.6f}, "
          f"max |dp| {dp.max():.3g}, status {int(a['status'])} / {int(b['status'])}", flush=True)
    for r in range(2):
        os.remove(f"{out}_{r}.npz")
