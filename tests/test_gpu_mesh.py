"""Mesh vertex update (PatchGeneration/Modules/Mesh.py:377-418): the device-built vertex->face
adjacency against igl's format (the numpy restatement vertex_triangle_adjacency, which matches the reference's
test_Mesh.py:145-150 arrays), and the fp32 kernel against the reference's fp64 run (mesh_update.npz)."""
import numpy as np
import pytest
import torch

import pcd_native as nat
from PatchGeneration.Modules.Mesh import Mesh, vertex_triangle_adjacency

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("out_dtype", [torch.int32, torch.int64])
def test_device_vta_matches_igl_format(golden, gpu, out_dtype):
    m = golden("mesh_update")
    f = m["f"].astype(np.int64)
    nv = len(m["v"]) + 3                                   # three trailing vertices of degree 0
    ref_vf, ref_ni = vertex_triangle_adjacency(f, nv)
    for fi in (torch.from_numpy(f), torch.from_numpy(f.astype(np.int32))):
        vf, ni = nat.mesh_vta(fi.to(gpu), nv, out_dtype=out_dtype)
        assert vf.dtype == out_dtype and ni.dtype == out_dtype
        np.testing.assert_array_equal(vf.cpu().numpy(), ref_vf)
        np.testing.assert_array_equal(ni.cpu().numpy(), ref_ni)


def test_device_vta_degenerate_and_bad_faces(gpu):
    f = np.array([[0, 1, 2], [2, 2, 3], [5, 0, 2]], np.int64)    # a face using one vertex twice; vertex 4 unused
    vf, ni = nat.mesh_vta(torch.from_numpy(f).to(gpu), 6)
    rvf, rni = vertex_triangle_adjacency(f, 6)
    np.testing.assert_array_equal(vf.cpu().numpy(), rvf)
    np.testing.assert_array_equal(ni.cpu().numpy(), rni)
    with pytest.raises(ValueError):
        nat.mesh_vta(torch.tensor([[0, 1, 9]], device=gpu), 6)


def test_mesh_update_fp32_matches_reference(golden, gpu):
    m = golden("mesh_update")
    bbox = float(np.linalg.norm(m["v"].max(0) - m["v"].min(0)))
    for k, key in ((1, "v_k1"), (15, "v_k15")):
        mesh = Mesh(m["v"].astype(np.float32), m["f"].astype(np.int64))
        mesh.updateVertices(m["n"].astype(np.float32), k=k, fp32=True)
        assert mesh.v.dtype == np.float32
        err = np.abs(mesh.v.astype(np.float64) - m[key]).max() / bbox
        assert err < 2e-6 * k, (k, err)
    # the fp64 path keeps its bitwise-level agreement with the device-built adjacency (test_gpu_parity covers k=1/15)
    mesh = Mesh(m["v"].copy(), m["f"].astype(np.int64))
    mesh.updateVertices(m["n"], k=15)
    np.testing.assert_allclose(mesh.v, m["v_k15"], rtol=0, atol=1e-10)
    vf, ni = mesh.getVertexTriangleAdjacency()
    rvf, rni = vertex_triangle_adjacency(m["f"], len(m["v"]))
    np.testing.assert_array_equal(vf, rvf)
    np.testing.assert_array_equal(ni, rni)
