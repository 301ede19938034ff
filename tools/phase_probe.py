"""Diagnostic (GPU box): the fused edge phase (k_phase, stage path) against the host build of step_edge on the
phase's own inputs, on the 200k headline sample with the oracle's f_n / positions / edge vectors injected."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normal-guided-pointcloud-denoiser_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pcd_native as nat  # noqa: E402
from oracle import pcd_oracle as O  # noqa: E402
from test_gpu_scale import bunny_cloud  # noqa: E402

dev = torch.device("cuda", 0)
K, KU = 32, 8
pos, nrm = bunny_cloud(200_000, 2, 0.005)
p0, n0 = pos.numpy(), nrm.numpy()
knn = O.FrozenKNN(p0)
d = 2 * O.mean_edge_length(p0, knn)
rec = {}
O.denoise_iteration(p0, n0, knn, d, K, KU, record=rec)
N = len(p0)
T = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
grid = nat.Grid(T(p0), k_hint=K)
fd = nat.FusedDenoiser(grid, K)
fd.load(T(p0), T(n0))
p = nat.make_params(k=K, k_update=KU, d=d)
perm = grid.perm().long()
rows = torch.arange(N, device=dev, dtype=torch.int32)
fd.stage(p, nat.STAGE_KNN_NVT1)
f4 = torch.zeros((N, 4), device=dev); f4[:, :3] = T(rec["f_n"])[perm]
fd.unpack(nat.FIELD_FN, rows, f4)
fd.stage(p, nat.STAGE_NVT2)
e4 = torch.zeros((N, 4), device=dev); e4[:, :3] = T(np.ascontiguousarray(rec["edge_vectors"]))[perm]
fd.unpack(nat.FIELD_EDGE, rows, e4)
red4 = torch.zeros(4, dtype=torch.float64, device=dev)
fd.stage(p, nat.STAGE_PHASE_SUM, 0, red4); fd.stage(p, nat.STAGE_PHASE_CENTRE, 0, red4)
fd.stage(p, nat.STAGE_PHASE_MAXDIST, 0, None); fd.stage(p, nat.STAGE_PHASE_APPLY, 0, None)
q4 = torch.zeros((N, 4), device=dev); q4[:, :3] = T(rec["pos_after_0"])[perm]
fd.unpack(nat.FIELD_POS, rows, q4)
# the phase's inputs as the device holds them (spatial order -> caller order)
inv = torch.empty_like(perm); inv[perm] = torch.arange(N, device=dev)
def field(f):
    x = fd.pack(f, rows)[:, :3]
    out = torch.empty_like(x); out[perm] = x
    return out.cpu().numpy()
pin, fn_d, edge_d = field(nat.FIELD_POS), field(nat.FIELD_FN), field(nat.FIELD_EDGE)
print("inputs == injected:", np.array_equal(pin, rec["pos_after_0"]), np.array_equal(fn_d, rec["f_n"]),
      np.array_equal(edge_d, np.ascontiguousarray(rec["edge_vectors"])))
fd.stage(p, nat.STAGE_PHASE_APPLY, 1, None)
got = field(nat.FIELD_POS)
fd.stage(p, nat.STAGE_FINISH)
cls = torch.empty(N, dtype=torch.int64, device=dev)
fd.store(None, None, cls)
cls = cls.cpu().numpy()
lists = fd.lists(K).cpu().numpy()
sel = np.nonzero(cls == 1)[0]
host = nat.host_step_csr(nat.STEP_EDGE, pin, fn_d, edge_d, sel, lists[sel, :KU], d, 0.2)
dv = np.abs(got[sel] - host).max(1)
print("device phase vs host step on the device's inputs: rows differ", int((dv > 0).sum()), "of", len(sel), "max", dv.max())
ok = (cls == rec["classes"]) & (lists[:, :KU] == rec["knn"][:, :KU]).all(1)
s2 = sel[ok[sel]]
dv2 = np.abs(got[s2] - rec["pos_after_1"][s2]).max(1)
print("device phase vs oracle (same class, same list):", int((dv2 > 0).sum()), "of", len(s2), "max", dv2.max())
h2 = nat.host_step_csr(nat.STEP_EDGE, rec["pos_after_0"], rec["f_n"], rec["edge_vectors"], s2, rec["knn"][s2, :KU], d, 0.2)
dv3 = np.abs(h2 - rec["pos_after_1"][s2]).max(1)
print("host on oracle inputs vs oracle:", int((dv3 > 0).sum()), "max", dv3.max())
