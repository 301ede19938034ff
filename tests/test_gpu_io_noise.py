"""Input synthesis ON THE DEVICE: Noise.generateNoise (Pointcloud/Modules/Noise.py:33-59)
and sampleObj's area-weighted barycentric sampling (Object.py:134-156) with HIP tensors and a device generator -- the
path bench.make_cloud takes for the 10M / 80M clouds.  The reference draws from torch's unseeded global RNG, so the
individual draws are "parity unpinned": the tests check the distributions the reference's code defines, as
tests/test_io_noise.py does on the CPU."""
import math
import os

import numpy as np
import pytest
import torch

from Pointcloud.Modules.GraphBuilder import GraphBuilder
from Pointcloud.Modules.Noise import Noise
from Pointcloud.Modules.Object import Pointcloud

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def graph_on(dev, n, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    pos = torch.rand((n, 3), generator=g, device=dev)
    nrm = torch.nn.functional.normalize(torch.randn((n, 3), generator=g, device=dev), dim=1)
    return GraphBuilder(Pointcloud(pos, nrm)).graph


def test_noise_on_device_along_normals(gpu):
    graph = graph_on(gpu, 1_000_000, 0)
    gt, nrm = graph.pos.clone(), graph.n.clone()
    l, level = 0.01, 0.3
    Noise(graph).generateNoise(level, l, generator=torch.Generator(device=gpu).manual_seed(1))
    assert graph.pos.device == gt.device                            # drawn and applied on the device
    off = (graph.pos - gt).double()
    along = (off * nrm.double()).sum(1)
    perp = off - along[:, None] * nrm.double()
    assert float(perp.abs().max()) < 1e-6
    sigma = l * level
    assert abs(float(along.std()) / sigma - 1) < 0.005
    assert abs(float(along.mean())) < 5 * sigma / math.sqrt(along.numel())
    kurt = float(((along - along.mean()) ** 4).mean() / along.var() ** 2)
    assert abs(kurt - 3) < 0.05
    assert not hasattr(graph, "n") and torch.equal(graph.gt, gt)


def test_noise_on_device_isotropic_and_impulsive(gpu):
    graph = graph_on(gpu, 1_000_000, 2)
    gt = graph.pos.clone()
    Noise(graph).generateNoise(0.5, 0.02, noise_direction=1, keepNormals=True,
                               generator=torch.Generator(device=gpu).manual_seed(3))
    sd = (graph.pos - gt).double().std(0)
    assert torch.allclose(sd, torch.full((3,), 0.01, dtype=torch.float64, device=gpu), rtol=0.005)
    n, level, l = 500_000, 0.3, 0.01
    graph = graph_on(gpu, n, 4)
    gt, nrm = graph.pos.clone(), graph.n.clone()
    Noise(graph).generateNoise(level, l, noise_type=1, generator=torch.Generator(device=gpu).manual_seed(5))
    # replay the generator: exactly int(n (1 - level)) offsets are dropped (Noise.py:55-57), the rest are the
    # Gaussian draws along the normals (an offset can still round to nothing in float32 by chance, so compare the
    # drawn offsets, not "position unchanged")
    g = torch.Generator(device=gpu).manual_seed(5)
    r = torch.randn((n, 3), generator=g, device=gpu) * (l * level)
    drop = torch.randperm(n, generator=g, device=gpu)[:int(n * (1 - level))]
    keep = torch.ones(n, dtype=torch.bool, device=gpu)
    keep[drop] = False
    assert int((~keep).sum()) == int(n * (1 - level))
    assert torch.equal(graph.pos[~keep], gt[~keep])
    assert torch.equal(graph.pos[keep], gt[keep] + nrm[keep] * r[keep, 0, None])


def test_sample_obj_on_device(gpu, tmp_path):
    """sampleObj(device=cuda) with a device generator: on-face samples, face normals, area-proportional hits."""
    fx = np.load(os.path.join(GOLDEN, "io.npz"))
    p = tmp_path / "fandisk.obj"
    with open(p, "w") as fh:
        for row in fx["v"]:
            fh.write("v " + " ".join(repr(float(x)) for x in row) + "\n")
        for row in fx["f"]:
            fh.write("f " + " ".join(str(int(x) + 1) for x in row) + "\n")
    n = 2_000_000
    pc = Pointcloud.sampleObj(str(p), n, device=gpu, generator=torch.Generator(device=gpu).manual_seed(0))
    assert pc.v.device.type == "cuda" and pc.v.shape == (n, 3) and pc.n.shape == (n, 3)
    # the same draws through sample_surface, keeping the face ids (sampleObj is exactly this call on the device)
    from Pointcloud.Modules.Object import sample_surface
    v32 = torch.from_numpy(fx["v"]).to(gpu)
    f = torch.from_numpy(fx["f"].astype(np.int64)).to(gpu)
    pos2, nrm2, fid = sample_surface(v32, f, n, generator=torch.Generator(device=gpu).manual_seed(0),
                                     return_faces=True)
    v = v32.double()
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    cr = torch.cross(b - a, c - a, dim=1)
    area = cr.norm(dim=1)
    fnrm = cr / area[:, None]
    d = ((pos2.double() - a[fid]) * fnrm[fid]).sum(1)
    assert float(d.abs().max()) < 1e-3 * float(area.max().sqrt())
    assert torch.allclose(nrm2.double(), fnrm[fid], atol=1e-5)
    # barycentric coordinates inside the triangle
    e0, e1, w = b[fid] - a[fid], c[fid] - a[fid], pos2.double() - a[fid]
    d00, d01, d11 = (e0 * e0).sum(1), (e0 * e1).sum(1), (e1 * e1).sum(1)
    d20, d21 = (w * e0).sum(1), (w * e1).sum(1)
    den = d00 * d11 - d01 * d01
    bv, bw = (d11 * d20 - d01 * d21) / den, (d00 * d21 - d01 * d20) / den
    assert float(bv.min()) > -1e-4 and float(bw.min()) > -1e-4 and float((bv + bw).max()) < 1 + 1e-4
    counts = torch.bincount(fid, minlength=len(f)).double()
    order = torch.argsort(area)
    for chunk in torch.tensor_split(order, 10):
        expect = float(area[chunk].sum() / area.sum() * n)
        got = float(counts[chunk].sum())
        assert abs(got - expect) < 5 * math.sqrt(expect) + 1, (got, expect)
    # sampleObj is this very call, and the inverse-CDF draws reproduce bit for bit (on the host too)
    assert torch.equal(pc.v, pos2) and torch.equal(pc.n, nrm2)
    assert torch.allclose(pc.n.norm(dim=1), torch.ones(1, device=gpu), atol=1e-5)


def test_bench_cloud_is_drawn_on_device(gpu):
    """bench.make_cloud (configs[3] / [4]): samples on the bunny surface plus N(0, (0.005 bbox)^2) per axis."""
    from bench import make_cloud
    pos, nrm, diag, surf = make_cloud(2_000_000, 2, gpu, clean=True)
    assert pos.device.type == "cuda" and surf.device.type == "cuda"
    # the same seed draws the same cloud again (every rank of a slab run and every bench process hold one cloud)
    pos2, nrm2, _ = make_cloud(2_000_000, 2, gpu)
    assert torch.equal(pos, pos2) and torch.equal(nrm, nrm2)
    off = (pos - surf).double()
    assert torch.allclose(off.std(0), torch.full((3,), 0.005 * diag, dtype=torch.float64, device=gpu), rtol=0.01)
    assert torch.allclose(nrm.norm(dim=1), torch.ones(1, device=gpu), atol=1e-5)
