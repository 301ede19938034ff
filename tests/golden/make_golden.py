"""Generate the golden fixtures under ``tests/golden/`` by running the REFERENCE Python hot path.

TEST INFRASTRUCTURE ONLY (build container).  Requires ``/root/reference`` and the in-container shims of
``refshim.py``.  Nothing here runs on the GPU box; the fixtures it writes are data
(inputs + the reference's outputs), committed as small ``.npz`` files.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only NAME]

Every fixture records which reference entry point produced it:
  fandisk_k32.npz   Processor.__init__/preprocess normals (GraphBuilder.py:60-63,77-82,99-111,129-209),
                    Selector.getKNNSelection (Selector.py:235-246), one Processor.denoise loop body at
                    k=32 staged per phase (Processor.py:119-139), iterates after 1/2/3/10 iterations in
                    fp32 and fp64, Chamfer to GT (Utils.py:253-265)
  fandisk_k16.npz   the same at Processor.denoise()'s default k=16 (Processor.py:110)
  fandisk_denoise.npz  Processor.denoise() verbatim (k=16, 2 iterations)
  steps.npz         Denoiser.{flat,edge,feature,corner,new,dummy}_step on fixed inputs (Denoiser.py:26-232),
                    Decompositionor.getBetterFilteredNVT + Decomposition.* (Decompositionor.py:57-106,278-300)
  lattice.npz       FeatureFix.ipynb lattice-cube known-answer test (n=9, 17; exact and 1e-4 jittered)
  mesh_update.npz   Mesh.updateVertices (PatchGeneration/Modules/Mesh.py:377-418) on the fandisk mesh
  metrics.npz       TorchUtils.ChamferDistance / PaperDistance / averageEdgeLength (Utils.py:253-299)
  until_min.npz     Processor.denoiseUntilMinimumError (Processor.py:141-185) on fandisk: strategy {0: flat_step,
                    1: edge_step, 2: feature_step}, k=8, alpha=[1, 0.2, 1], d=2l, error PaperDistance; the returned
                    pos / errors / iteration count and the error trajectory
  thesis.npz        the thesis driver "Ours" (PostProcessing.ipynb:1069-1090) on fandisk: 2 iterations, Jacobi
                    across classes, flat_step + feature_step at d*20000, global clamp ||temp_pos - original_pos|| < d
  cpsd.npz          the CPSD ("Martin") path: radius selections, normal-filtered NVT / PVT, VU features, corner_step,
                    getVUDecomposition, and 2 iterations of the notebook's 50-iteration driver (PostProcessing.ipynb
                    :1041-1062, j == 1) verbatim: positions, normals, classes and clamp mask per iteration
  io.npz            Object.Pointcloud.loadObj readback of models/fandisk.obj (Object.py:71-89)
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()
sys.path.insert(0, REF)
from Pointcloud.Modules.Object import Pointcloud  # noqa: E402
from Pointcloud.Modules.Processor import Processor  # noqa: E402
from Pointcloud.Modules.Utils import TorchUtils  # noqa: E402
from PatchGeneration.Modules.Mesh import Mesh  # noqa: E402

torch.set_num_threads(8)


def run_with_big_stack(fn, *a):
    """flipNormalsWithMST is a recursive DFS (GraphBuilder.py:191-202): give it room."""
    sys.setrecursionlimit(10 ** 6)
    threading.stack_size(512 * 1024 * 1024)
    out = {}

    def target():
        out["r"] = fn(*a)

    t = threading.Thread(target=target)
    t.start()
    t.join()
    return out.get("r")


def ref_normals(processor, k=12, flip=True):
    g = processor.graph
    g.edge_index = processor.graphBuilder.getKNNEdgeIndex(k)
    run_with_big_stack(processor.graphBuilder.setAndFlipNormals, flip)
    return g.n.clone()


def load_obj(path, dtype=torch.float32):
    v, f = refshim.read_obj(path)
    return torch.tensor(v, dtype=dtype), f


def chamfer_mean(a, b):
    return float(TorchUtils.ChamferDistance(a, b).mean())


def denoise_body(proc, k, k_u, d, alphas=(1, 0.2, 1), angle=None, record=None):
    """One iteration of Processor.denoise's loop body (Processor.py:124-139) with k / k_u exposed."""
    dec, f_n = proc.getMyFeatureDecomposition(k, angle)
    classes = dec.getClasses()
    sel = proc.selector.getKNNSelection(k_u)
    if record is not None:
        record["classes"] = classes.clone()
        record["f_n"] = f_n.clone()
        record["eigval2"] = dec.eigval.clone()
        record["eigvec2"] = dec.eigvec.clone()
        record["knn_u"] = sel.j.view(-1, k_u).clone()
    for key in range(3):
        idx = (classes == key).nonzero().flatten()
        if idx.size(0) == 0:
            if record is not None:
                record[f"pos_after_{key}"] = proc.graph.pos.clone()
            continue
        if key == 0:
            new_pos = proc.denoiser.flat_step(sel.filter(idx), f_n, d, alphas[key])
        elif key == 1:
            new_pos = proc.denoiser.edge_step(sel.filter(idx), f_n, dec.eigvec[..., 0], d, alphas[key])
        else:
            new_pos = proc.denoiser.feature_step(sel.filter(idx), f_n, d, alphas[key])
        proc.graph.pos[idx] = new_pos
        if record is not None:
            record[f"pos_after_{key}"] = proc.graph.pos.clone()
    proc.graph.n = f_n


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def gen_fandisk(out_dir, k=32):
    """fandisk_k{k}.npz: the frozen-snapshot kNN, NVT1 and one Processor.denoise loop body at feature-kNN size k
    staged per phase, the iterates after 1/2/3/10 iterations (fp32 and fp64).  k = 32 is the metric's size; k = 16 is
    Processor.denoise()'s own default (Processor.py:110).  The k = 32 call also writes fandisk_denoise.npz."""
    t0 = time.time()
    pos, faces = load_obj(f"{REF}/models/fandisk_gaus_n6_noisy.obj")
    gt, _ = load_obj(f"{REF}/models/fandisk.obj")
    N = pos.size(0)
    pc = Pointcloud(pos.clone())
    proc = Processor(pc)
    n0 = ref_normals(proc)
    pos0 = proc.graph.pos.clone()
    res = {"pos0": np32(pos0), "n0": np32(n0), "gt": np32(gt)}
    # frozen-snapshot kNN (Selector.py:141,243) incl. scipy f64 distances
    dist, idx = proc.selector.kdtree.query(pos0.numpy(), k=k)
    res[f"knn{k}"] = idx.astype(np.int32)
    res[f"knn{k}_d"] = dist.astype(np.float64)
    sel6 = proc.selector.getKNNSelection(6)
    l = TorchUtils.averageEdgeLength(proc.graph.pos, sel6.getEdgeIndex())
    d = float(2 * l)
    res["l"] = np.float64(l)
    res["d"] = np.float64(d)
    # Stage-by-stage NVT1 (Processor.getMyFeatureDecomposition, Processor.py:110-117) at k
    angle = torch.pi * 5 / 12
    sel = proc.selector.getKNNSelection(k)
    nvt1 = proc.decompositionor.getBetterFilteredNVT(sel, proc.graph.n, angle)
    res["eigval1"] = np32(nvt1.eigval)
    res["eigvec1"] = np32(nvt1.eigvec)
    rec = {}
    denoise_body(proc, k, 8, d, record=rec)
    for k_, v_ in rec.items():
        res["it1_" + k_] = v_.numpy() if v_.dtype in (torch.int64, torch.int32) else np32(v_)
    cds = [chamfer_mean(gt, pos0)]
    iters = {1: np32(proc.graph.pos)}
    norms = {1: np32(proc.graph.n)}
    cds.append(chamfer_mean(gt, proc.graph.pos))
    for it in range(2, 11):
        denoise_body(proc, k, 8, d)
        cds.append(chamfer_mean(gt, proc.graph.pos))
        if it in (2, 3, 10):
            iters[it] = np32(proc.graph.pos)
            norms[it] = np32(proc.graph.n)
    for it in iters:
        res[f"pos_it{it}"] = iters[it]
        res[f"n_it{it}"] = norms[it]
    res["cd_f32"] = np.asarray(cds)
    # fp64 run of the same loop (divergence envelope)
    pc64 = Pointcloud(pos0.double().clone(), n0.double().clone())
    p64 = Processor(pc64)
    cds64 = [chamfer_mean(gt.double(), pos0.double())]
    for it in range(1, 11):
        denoise_body(p64, k, 8, d)
        cds64.append(chamfer_mean(gt.double(), p64.graph.pos))
        if it in (1, 2, 3, 10):
            res[f"pos64_it{it}"] = p64.graph.pos.numpy().astype(np.float64)
    res["cd_f64"] = np.asarray(cds64)
    res["k"] = np.int64(k)
    np.savez_compressed(os.path.join(out_dir, f"fandisk_k{k}.npz"), **res)
    print(f"fandisk_k{k}: N={N} d={d:.5f} CD {cds[0]:.4g} -> {cds[1]:.4g} {cds[2]:.4g} {cds[3]:.4g} .. {cds[-1]:.4g}"
          f"  ({time.time()-t0:.1f}s)")
    if k != 32:
        return

    # Processor.denoise() verbatim (k=16, k_u=8, 2 iterations)
    pc2 = Pointcloud(pos0.clone(), n0.clone())
    p2 = Processor(pc2)
    p2.denoise()
    np.savez_compressed(os.path.join(out_dir, "fandisk_denoise.npz"), pos0=np32(pos0), n0=np32(n0),
                        pos=np32(p2.graph.pos), n=np32(p2.graph.n), alias_ok=np.int8(p2.graph.pos is pc2.v))
    print("fandisk_denoise done")


def gen_steps(out_dir):
    """Single-step kernels fed identical inputs (per-kernel parity)."""
    f = np.load(os.path.join(out_dir, "fandisk_k32.npz"))
    pos0 = torch.from_numpy(f["pos0"])
    n0 = torch.from_numpy(f["n0"])
    pc = Pointcloud(pos0.clone(), n0.clone())
    proc = Processor(pc)
    res = {"pos": f["pos0"], "n": f["n0"]}
    g = torch.Generator().manual_seed(7)
    # second normal field, a rotated perturbation (so f_n-like inputs differ from n0)
    n1 = torch.nn.functional.normalize(n0 + 0.05 * torch.randn(n0.shape, generator=g), dim=1)
    res["n1"] = np32(n1)
    for rho_name, rho in (("a5pi12", torch.pi * 5 / 12), ("api3", torch.pi / 3)):
        for k in (8, 16):
            sel = proc.selector.getKNNSelection(k)
            dec = proc.decompositionor.getBetterFilteredNVT(sel, n1, rho)
            res[f"nvt_{rho_name}_k{k}_eigval"] = np32(dec.eigval)
            res[f"nvt_{rho_name}_k{k}_eigvec"] = np32(dec.eigvec)
            res[f"nvt_{rho_name}_k{k}_classes"] = dec.getClasses().numpy()
            pl, li, sp = dec.getNVTFeatures()
            res[f"nvt_{rho_name}_k{k}_features"] = np32(torch.stack([pl, li, sp], 1))
            res[f"nvt_{rho_name}_k{k}_vu"] = np32(dec.getVUSmoothedNormals(n1))
            res[f"knn{k}"] = sel.j.view(-1, k).numpy().astype(np.int32)
    sel8 = proc.selector.getKNNSelection(8)
    dec = proc.decompositionor.getBetterFilteredNVT(proc.selector.getKNNSelection(16), n1, torch.pi * 5 / 12)
    ev = dec.eigvec[..., 0]
    res["edge_vectors"] = np32(ev)
    gsel = torch.Generator().manual_seed(11)
    idx = torch.randperm(pos0.size(0), generator=gsel)[:2000].sort().values
    res["subset"] = idx.numpy().astype(np.int64)
    d = float(f["d"])
    for alpha in (1.0, 0.2):
        s = sel8.filter(idx)
        tag = f"a{alpha}"
        res[f"flat_{tag}"] = np32(proc.denoiser.flat_step(s, n1, d, alpha))
        res[f"edge_{tag}"] = np32(proc.denoiser.edge_step(s, n1, ev, d, alpha))
        res[f"feature_{tag}"] = np32(proc.denoiser.feature_step(s, n1, d, alpha))
        res[f"corner_{tag}"] = np32(proc.denoiser.corner_step(s, n1, d, alpha))
        res[f"new_{tag}"] = np32(proc.denoiser.new_step(s, n1, d, alpha))
        res[f"dummy_{tag}"] = np32(proc.denoiser.dummy_step(s, n1, d, alpha))
        # unclamped variants (d huge) isolate the solve from the clamp decision
        res[f"edge_{tag}_noclamp"] = np32(proc.denoiser.edge_step(s, n1, ev, 1e9, alpha))
        res[f"feature_{tag}_noclamp"] = np32(proc.denoiser.feature_step(s, n1, 1e9, alpha))
        res[f"corner_{tag}_noclamp"] = np32(proc.denoiser.corner_step(s, n1, 1e9, alpha))
        res[f"flat_{tag}_noclamp"] = np32(proc.denoiser.flat_step(s, n1, 1e9, alpha))
    res["d"] = np.float64(d)
    # PCA normals without orientation (GraphBuilder.getPVTDecompositionWithKNN, GraphBuilder.py:99-111)
    ei = proc.graphBuilder.getKNNEdgeIndex(12)
    res["knn12_noself"] = ei[1].view(-1, 12).numpy().astype(np.int32)
    res["pca_n"] = np32(proc.graphBuilder.getPVTDecompositionWithKNN(ei)[..., 0])
    np.savez_compressed(os.path.join(out_dir, "steps.npz"), **res)
    print("steps done")


def lattice(n):
    t = torch.linspace(-1, 1, n)
    x, y, z = torch.meshgrid(t, t, t, indexing="ij")
    p = torch.stack([x, y, z], -1).view(-1, 3)
    keep = (p.abs() == 1).any(1)
    return p[keep].contiguous()


def gen_lattice(out_dir):
    res = {}
    for n in (9, 17):
        for jit in (0.0, 1e-4):
            pos = lattice(n)
            gt_c = pos.square().to(torch.int).sum(1) - 1  # FeatureFix.ipynb:59 (0 flat, 1 edge, 2 corner)
            if jit:
                pos = pos + jit * torch.randn(pos.shape, generator=torch.Generator().manual_seed(n))
            proc = Processor(Pointcloud(pos.clone()))
            nrm = ref_normals(proc)
            dec, f_n = proc.getMyFeatureDecomposition()
            cls = dec.getClasses()
            tag = f"n{n}_j{int(jit > 0)}"
            res[f"{tag}_pos"] = np32(pos)
            res[f"{tag}_n"] = np32(nrm)
            res[f"{tag}_classes"] = cls.numpy()
            res[f"{tag}_gt"] = gt_c.numpy()
            res[f"{tag}_fn"] = np32(f_n)
            res[f"{tag}_eigval"] = np32(dec.eigval)
            acc = float((cls == gt_c).float().mean())
            res[f"{tag}_acc"] = np.float64(acc)
            print(f"lattice {tag}: N={pos.size(0)} acc={acc*100:.2f}%")
    np.savez_compressed(os.path.join(out_dir, "lattice.npz"), **res)


def vta_of(f, V):
    flat = f.reshape(-1)
    order = np.argsort(flat, kind="stable")
    VF = (order // 3).astype(np.int64)
    counts = np.bincount(flat, minlength=V)
    NI = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return VF, NI


def gen_mesh(out_dir):
    vn, f = refshim.read_obj(f"{REF}/models/fandisk_gaus_n6_noisy.obj")
    vc, fc = refshim.read_obj(f"{REF}/models/fandisk.obj")
    assert (f == fc).all()
    clean = Mesh(vc.copy(), fc, f2f=np.zeros(1), vta=vta_of(fc, len(vc)))
    n = clean.getFaceNormals()  # Mesh.py:110-114
    mesh = Mesh(vn.copy(), f, f2f=np.zeros(1), vta=vta_of(f, len(vn)))
    v_in = mesh.v.copy()
    t0 = time.time()
    mesh.updateVertices(n, k=15)
    dt = (time.time() - t0) / 15
    m1 = Mesh(vn.copy(), f, f2f=np.zeros(1), vta=vta_of(f, len(vn)))
    m1.updateVertices(n, k=1)
    np.savez_compressed(os.path.join(out_dir, "mesh_update.npz"), v=v_in, f=f.astype(np.int32), n=n,
                        v_k15=mesh.v, v_k1=m1.v, vc=vc, s_per_iter=np.float64(dt))
    print(f"mesh_update: V={len(vn)} F={len(f)} {dt*1e3:.1f} ms/iter; MSE vs clean {np.mean((mesh.v-vc)**2):.3e}")


def gen_metrics(out_dir):
    f = np.load(os.path.join(out_dir, "fandisk_k32.npz"))
    g = torch.Generator().manual_seed(3)
    a = torch.from_numpy(f["gt"])[torch.randperm(6475, generator=g)[:1000]]
    b = torch.from_numpy(f["pos0"])[torch.randperm(6475, generator=g)[:1200]]
    cd = TorchUtils.ChamferDistance(a, b)
    pdist = TorchUtils.PaperDistance(a, b)
    hd = TorchUtils.HausdorffDistance(a, b)
    proc = Processor(Pointcloud(b.clone()))
    ael = TorchUtils.averageEdgeLength(b, proc.selector.getKNNSelection(6).getEdgeIndex())
    np.savez_compressed(os.path.join(out_dir, "metrics.npz"), a=np32(a), b=np32(b), chamfer=np32(cd),
                        paper=np32(pdist), hausdorff=np32(hd), avg_edge_len=np.float64(ael))
    print(f"metrics: CD mean {float(cd.mean()):.4g}")


def gen_cpsd(out_dir):
    """The CPSD ("Martin") feature path: radius selection (Selector.py:214-233, scipy query_ball_point on the frozen
    f64 snapshot), getNormalFilteredNVT (Decompositionor.py:260-276), VU smoothing, getNormalFilteredPVT
    (Decompositionor.py:172-211), getVUFeatures (:84-85), as composed by Processor.getMartinFeatureDecomposition
    (Processor.py:102-108) and Processor.getVUDecomposition (Processor.py:83-100); plus corner_step on the CPSD
    classes (the PostProcessing.ipynb:1041-1062 driver's corner phase)."""
    f = np.load(os.path.join(out_dir, "fandisk_k32.npz"))
    pos0 = torch.from_numpy(f["pos0"])
    n0 = torch.from_numpy(f["n0"])
    d = float(f["d"])
    res = {"pos": f["pos0"], "n": f["n0"], "d": np.float64(d)}
    proc = Processor(Pointcloud(pos0.clone(), n0.clone()))
    for tag, r in (("r1", d), ("r2", 2 * d)):
        sel = proc.selector.getPointsInRangeSelection(r)
        res[f"sel_{tag}_radius"] = np.float64(r)
        res[f"sel_{tag}_slices"] = sel.slices.numpy().astype(np.int64)
        res[f"sel_{tag}_j"] = sel.j.numpy().astype(np.int32)
    dec, fn = proc.getMartinFeatureDecomposition(r=d)
    sel = proc.selector.getPointsInRangeSelection(d)
    nvt = proc.decompositionor.getNormalFilteredNVT(sel, n0, 0.9)
    res["nvt_eigval"] = np32(nvt.eigval)
    res["nvt_eigvec"] = np32(nvt.eigvec)
    res["f_n"] = np32(fn)
    res["pvt_eigval"] = np32(dec.eigval)
    res["pvt_eigvec"] = np32(dec.eigvec)
    res["vu_classes"] = dec.getVUFeatures(tau=0.3).numpy().astype(np.int64)
    sel8 = proc.selector.getKNNSelection(8)
    corners = (dec.getVUFeatures(tau=0.3) == 2).nonzero().flatten()
    res["corner_idx"] = corners.numpy().astype(np.int64)
    res["corner_pos"] = np32(proc.denoiser.corner_step(sel8.filter(corners), fn, d * 20000, 1.0))
    # Processor.getVUDecomposition: r = 2 * mean kNN(6, self excluded) edge length, rho = 0.95 for both votes
    vu = proc.getVUDecomposition()
    res["vud_eigval"] = np32(vu.eigval)
    res["vud_eigvec"] = np32(vu.eigvec)
    # the CPSD driver itself: PostProcessing.ipynb:1041-1062 (j == 1, "Martin") verbatim for 2 of its 50
    # iterations on fandisk -- radius decomposition, VU classes, flat / edge / corner steps at d*20000 (Jacobi across
    # classes through temp_pos), the global clamp ||temp_pos - original_pos|| < d, n := f_n
    col_value = Processor(Pointcloud(pos0.clone(), n0.clone()))
    l = TorchUtils.averageEdgeLength(col_value.graph.pos, col_value.selector.getKNNSelection(6).getEdgeIndex())
    dd = 2 * l
    original_pos = col_value.graph.pos.clone()
    res["drv_d"] = np.float64(dd)
    alphas = [0.1, 1, 1]
    for it in range(2):
        decomposition, f_n = col_value.getMartinFeatureDecomposition(r=dd)
        classes = decomposition.getVUFeatures(tau=0.3)
        selection = col_value.selector.getKNNSelection(k=8)
        temp_pos = col_value.graph.pos.clone()
        for key in range(3):
            indices = (classes == key).nonzero().flatten()
            if indices.size(0) == 0:
                continue
            elif key == 0:
                new_pos = col_value.denoiser.flat_step(selection.filter(indices), f_n, dd * 20000, alphas[key])
            elif key == 1:
                edge_vectors = decomposition.eigvec[..., 0]
                new_pos = col_value.denoiser.edge_step(selection.filter(indices), f_n, edge_vectors, dd * 20000,
                                                       alphas[key])
            else:
                new_pos = col_value.denoiser.corner_step(selection.filter(indices), f_n, dd * 20000, alphas[key])
            temp_pos[indices] = new_pos
        mask = (temp_pos - original_pos).norm(dim=1) < dd
        col_value.graph.pos[mask] = temp_pos[mask]
        col_value.graph.n = f_n
        res[f"drv_pos_it{it + 1}"] = np32(col_value.graph.pos)
        res[f"drv_n_it{it + 1}"] = np32(col_value.graph.n)
        res[f"drv_classes_it{it + 1}"] = classes.numpy().astype(np.int64)
        res[f"drv_mask_it{it + 1}"] = mask.numpy()
    np.savez_compressed(os.path.join(out_dir, "cpsd.npz"), **res)
    lens = np.diff(res["sel_r1_slices"])
    print(f"cpsd: r={d:.5f} neighbours/pt {lens.mean():.1f} (min {lens.min()}, max {lens.max()}), "
          f"VU classes {np.bincount(res['vu_classes'], minlength=3)}, corners {len(corners)}")


def gen_until_min(out_dir):
    f = np.load(os.path.join(out_dir, "fandisk_k32.npz"))
    pos0 = torch.from_numpy(f["pos0"])
    n0 = torch.from_numpy(f["n0"])
    gt = torch.from_numpy(f["gt"])
    pc = Pointcloud(pos0.clone(), n0.clone())
    proc = Processor(pc)
    l = TorchUtils.averageEdgeLength(proc.graph.pos, proc.selector.getKNNSelection(6).getEdgeIndex())
    d = float(2 * l)
    traj = []

    def err(gt_pos, pos):
        e = TorchUtils.PaperDistance(gt_pos, pos)
        traj.append(float(e.mean()))
        return e

    den = proc.denoiser
    strategy = {0: den.flat_step, 1: den.edge_step, 2: den.feature_step}
    pos, errors, iters = proc.denoiseUntilMinimumError(gt, strategy, k=8, alpha=[1, 0.2, 1], d=d, error_funcs=[err])
    np.savez_compressed(os.path.join(out_dir, "until_min.npz"), pos0=f["pos0"], n0=f["n0"], gt=f["gt"],
                        d=np.float64(d), pos=np32(pos), errors=np32(errors[0]), iterations=np.int64(iters),
                        trajectory=np.asarray(traj), pc_v=np32(pc.v), graph_pos=np32(proc.graph.pos))
    print(f"until_min: d={d:.5f} iterations={iters} error trajectory {['%.4g' % x for x in traj]}")


def gen_thesis(out_dir):
    """PostProcessing.ipynb:1069-1090 (j == 3, "Ours") verbatim on fandisk."""
    f = np.load(os.path.join(out_dir, "fandisk_k32.npz"))
    col_value = Processor(Pointcloud(torch.from_numpy(f["pos0"]).clone(), torch.from_numpy(f["n0"]).clone()))
    l = TorchUtils.averageEdgeLength(col_value.graph.pos, col_value.selector.getKNNSelection(6).getEdgeIndex())
    d = 2 * l
    original_pos = col_value.graph.pos.clone()
    res = {"pos0": f["pos0"], "n0": f["n0"], "d": np.float64(d)}
    alphas = [1, 0.2, 1]
    for it in range(2):
        decomposition, f_n = col_value.getMyFeatureDecomposition()
        classes = decomposition.getClasses()
        selection = col_value.selector.getKNNSelection(8)
        temp_pos = col_value.graph.pos.clone()
        for key in range(3):
            indices = (classes == key).nonzero().flatten()
            if indices.size(0) == 0:
                continue
            elif key == 0:
                new_pos = col_value.denoiser.flat_step(selection.filter(indices), f_n, d * 20000, alphas[key])
            else:
                new_pos = col_value.denoiser.feature_step(selection.filter(indices), f_n, d * 20000, alphas[key])
            temp_pos[indices] = new_pos
        mask = (temp_pos - original_pos).norm(dim=1) < d
        col_value.graph.pos[mask] = temp_pos[mask]
        col_value.graph.n = f_n
        res[f"pos_it{it + 1}"] = np32(col_value.graph.pos)
        res[f"n_it{it + 1}"] = np32(col_value.graph.n)
        res[f"classes_it{it + 1}"] = classes.numpy()
        res[f"mask_it{it + 1}"] = mask.numpy()
    np.savez_compressed(os.path.join(out_dir, "thesis.npz"), **res)
    print(f"thesis: d={float(d):.5f} masked-out after 2 iterations: {int((~res['mask_it2']).sum())}")


def gen_io(out_dir):
    """Pointcloud.loadObj (Object.py:71-89) on models/fandisk.obj: the vertex array the reference reads (igl is
    absent here: refshim's OBJ reader stands in for igl.read_triangle_mesh, so this pins the readback of the file's
    `v` lines and the face count)."""
    v, faces = refshim.read_obj(f"{REF}/models/fandisk.obj")
    np.savez_compressed(os.path.join(out_dir, "io.npz"), v=np.asarray(v, np.float32), f=np.asarray(faces, np.int32))
    print(f"io: fandisk.obj V={len(v)} F={len(faces)}")


GENS = {"fandisk": gen_fandisk, "fandisk16": lambda out_dir: gen_fandisk(out_dir, 16), "steps": gen_steps, "lattice": gen_lattice, "mesh": gen_mesh,
        "metrics": gen_metrics, "cpsd": gen_cpsd, "until_min": gen_until_min, "thesis": gen_thesis, "io": gen_io}

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    torch.manual_seed(0)
    for name, fn in GENS.items():
        if args.only and name not in args.only.split(","):
            continue
        fn(HERE)
