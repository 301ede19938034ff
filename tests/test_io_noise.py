"""Input synthesis and I/O on the CPU: Noise.generateNoise statistics
(Pointcloud/Modules/Noise.py:33-59), Pointcloud.loadObj against the reference's readback of models/fandisk.obj
(Object.py:71-89; fixture tests/golden/io.npz), saveObj/loadObj round trip, and sampleObj's area-weighted
barycentric sampling (Object.py:134-156).

The reference draws its noise from torch's unseeded global RNG, so no fixture can pin the offsets themselves: the
tests check the distribution the reference's code defines (sigma = level x mean edge length, offsets along the
normal or isotropic, an impulsive fraction of exactly int(N (1 - level)) zero offsets) -- "parity unpinned" for the
individual random draws.
"""
import math
import os

import numpy as np
import pytest
import torch

from Pointcloud.Modules.GraphBuilder import GraphBuilder
from Pointcloud.Modules.Noise import Noise
from Pointcloud.Modules.Object import Pointcloud, read_obj_arrays, sample_surface

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def graph_of(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand((n, 3), generator=g)
    nrm = torch.nn.functional.normalize(torch.randn((n, 3), generator=g), dim=1)
    return GraphBuilder(Pointcloud(pos, nrm)).graph


def test_noise_gaussian_along_normals():
    graph = graph_of(200_000)
    gt, nrm = graph.pos.clone(), graph.n.clone()
    l, level = 0.01, 0.3
    Noise(graph).generateNoise(level, l, generator=torch.Generator().manual_seed(1))
    off = graph.pos - gt
    along = (off * nrm).sum(1)
    perp = off - along[:, None] * nrm
    assert float(perp.abs().max()) < 1e-6                      # direction 0: offsets along the vertex normal
    sigma = l * level
    assert abs(float(along.std()) / sigma - 1) < 0.01          # sigma = mean edge length x level
    assert abs(float(along.mean())) < 5 * sigma / math.sqrt(len(along))
    kurt = float(((along - along.mean()) ** 4).mean() / along.var() ** 2)
    assert abs(kurt - 3) < 0.1                                  # Gaussian
    assert torch.equal(graph.gt, gt) and torch.equal(graph.gt_n, nrm)
    assert not hasattr(graph, "n")                              # normals dropped (keepNormals=False)


def test_noise_random_direction_and_keep_normals():
    graph = graph_of(200_000, 2)
    gt = graph.pos.clone()
    Noise(graph).generateNoise(0.5, 0.02, noise_direction=1, keepNormals=True,
                               generator=torch.Generator().manual_seed(3))
    off = graph.pos - gt
    sd = off.std(0)
    assert torch.allclose(sd, torch.full((3,), 0.01), rtol=0.01)   # isotropic, per-axis sigma
    assert abs(float(torch.corrcoef(off.T)[0, 1])) < 0.01
    assert hasattr(graph, "n")


def test_noise_impulsive_fraction():
    n, level = 100_000, 0.3
    graph = graph_of(n, 4)
    gt, nrm = graph.pos.clone(), graph.n.clone()
    Noise(graph).generateNoise(level, 0.01, noise_type=1, generator=torch.Generator().manual_seed(5))
    # replay the generator: exactly int(n (1 - level)) offsets zeroed (Noise.py:55-57), the rest the Gaussian draws
    g = torch.Generator().manual_seed(5)
    r = torch.randn((n, 3), generator=g) * (0.01 * level)
    drop = torch.randperm(n, generator=g)[:int(n * (1 - level))]
    keep = torch.ones(n, dtype=torch.bool)
    keep[drop] = False
    assert int((~keep).sum()) == int(n * (1 - level))
    assert torch.equal(graph.pos[~keep], gt[~keep])
    assert torch.equal(graph.pos[keep], gt[keep] + nrm[keep] * r[keep, 0, None])


def test_noise_rejects_out_of_range_and_resets():
    graph = graph_of(100)
    noise = Noise(graph)
    for kw in ({"noise_level": 1.5}, {"noise_level": -0.1}, {"noise_level": 0.1, "noise_type": 2},
               {"noise_level": 0.1, "noise_direction": -1}):
        args = dict(mean_edge_length=1.0, **kw)
        with pytest.raises(ValueError):
            noise.generateNoise(**args)
    with pytest.raises(ValueError):
        noise.resetNoise()                                      # never applied
    gt = graph.pos.clone()
    noise.generateNoise(0.2, 1.0, keepNormals=True, generator=torch.Generator().manual_seed(0))
    noise.resetNoise()
    assert torch.equal(graph.pos, gt)


def _write_obj(path, v, f):
    with open(path, "w") as fh:
        fh.write("# fixture written from tests/golden/io.npz\n")
        for row in v:
            fh.write("v " + " ".join(repr(float(x)) for x in row) + "\n")
        for row in f:
            fh.write("f " + " ".join(str(int(x) + 1) for x in row) + "\n")


def test_load_obj_matches_reference_readback(tmp_path):
    """io.npz holds the vertex / face arrays the reference's loader reads from models/fandisk.obj (make_golden.py
    gen_io); an OBJ written from them must load back to exactly those float32 vertices and faces."""
    fx = np.load(os.path.join(GOLDEN, "io.npz"))
    p = tmp_path / "fandisk.obj"
    _write_obj(p, fx["v"], fx["f"])
    pc = Pointcloud.loadObj(str(p))
    assert pc.v.dtype == torch.float32 and pc.v.shape == (6475, 3)
    np.testing.assert_array_equal(pc.v.numpy(), fx["v"])
    v, _, fv, _ = read_obj_arrays(str(p))
    np.testing.assert_array_equal(fv, fx["f"].astype(np.int64))
    assert pc.file_path == str(p)


def test_save_obj_round_trip(tmp_path):
    g = torch.Generator().manual_seed(9)
    v = torch.randn((500, 3), generator=g)
    n = torch.nn.functional.normalize(torch.randn((500, 3), generator=g), dim=1)
    p = tmp_path / "cloud.obj"
    Pointcloud(v, n).saveObj(str(p))
    back = Pointcloud.loadObj(str(p))
    assert torch.equal(back.v, v) and torch.equal(back.n, n)
    with pytest.raises(FileExistsError):                       # the reference opens with mode "x" (Object.py:58-69)
        Pointcloud(v).saveObj(str(p))


def test_sample_obj_area_weighted(tmp_path):
    """Samples lie on their mesh's faces, carry the face normal, and hit each face in proportion to its area."""
    fx = np.load(os.path.join(GOLDEN, "io.npz"))
    p = tmp_path / "fandisk.obj"
    _write_obj(p, fx["v"], fx["f"])
    n = 400_000
    pc = Pointcloud.sampleObj(str(p), n, generator=torch.Generator().manual_seed(0))
    v = torch.from_numpy(fx["v"])
    f = torch.from_numpy(fx["f"].astype(np.int64))
    pos, nrm, fid = sample_surface(v, f, n, generator=torch.Generator().manual_seed(0), return_faces=True)
    assert torch.equal(pos, pc.v) and torch.equal(nrm, pc.n)
    v = v.double()
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    cr = torch.cross(b - a, c - a, dim=1)
    area = cr.norm(dim=1)
    # on the face plane, inside the triangle (barycentric coordinates >= 0)
    fn = cr[fid] / area[fid, None]
    d = ((pc.v.double() - a[fid]) * fn).sum(1)
    assert float(d.abs().max()) < 1e-3 * float(area.max().sqrt())
    assert torch.allclose(pc.n.double(), fn, atol=1e-5)
    # face hit frequency vs area share, aggregated over area deciles (chi-square-sized tolerance)
    counts = torch.bincount(fid, minlength=len(f)).double()
    order = torch.argsort(area)
    for chunk in torch.tensor_split(order, 10):
        expect = float(area[chunk].sum() / area.sum() * n)
        got = float(counts[chunk].sum())
        assert abs(got - expect) < 5 * math.sqrt(expect) + 1, (got, expect)
