"""Graph construction and initial normals (drop-in for Pointcloud/Modules/GraphBuilder.py, hot-path subset).

getKNNEdgeIndex(k) -> kNN of the CURRENT positions over a fresh grid, self excluded (torch_cluster.knn_graph,
flow="target_to_source", GraphBuilder.py:60-63); getPVTDecompositionWithKNN -> pcd_pca_dense (covariance about the
neighbours' mean + the LAPACK-ssyevd 3x3 eigh, :99-111); flipNormals -> pcd_orient_normals_mst_gpu (Borůvka MST + Euler-tour
rooting + sign pointer jumping on the device, :129-209; bit-identical to the host Kruskal + DFS pcd_orient_normals_mst,
which the tests keep as the cross-check).
"""
from __future__ import annotations

import torch

import pcd_native as _nat
from .Graph import Data
from .Object import Pointcloud
from .Utils import GeneralUtils, TorchUtils


class GraphBuilder:

    def __init__(self, pointcloud: Pointcloud):
        GeneralUtils.validateAttributes(pointcloud, ["v"])
        self.device = pointcloud.v.device
        self.pointcloud = pointcloud
        self.graph = Data(pos=pointcloud.v)          # alias of the caller's tensor (GraphBuilder.py:50)
        if pointcloud.hasNormals():
            self.graph.n = pointcloud.n

    def getKNNEdgeIndex(self, k: int = 12) -> torch.Tensor:
        _graph = self.graph
        GeneralUtils.validateAttributes(_graph, ["pos"])
        pos = _graph.pos
        grid = _nat.Grid(pos, k_hint=k + 1)
        nbr = grid.knn(pos, k, exclude_self=True)
        n = pos.size(0)
        row = torch.arange(n, device=nbr.device).repeat_interleave(k)
        return torch.stack([row, nbr.reshape(-1)]).to(pos.device)

    def setAndFlipNormals(self, flip: bool = True) -> None:
        GeneralUtils.validateAttributes(self.graph, ["edge_index"])
        self.setPVTNormals(self.graph.edge_index)
        if flip:
            self.flipNormals()

    def setPVTNormals(self, edge_index: torch.Tensor) -> None:
        eigvec = self.getPVTDecompositionWithKNN(edge_index)
        self.graph.n = eigvec[..., 0]

    def getPVTDecompositionWithKNN(self, edge_index: torch.Tensor) -> torch.Tensor:
        _graph = self.graph
        GeneralUtils.validateAttributes(_graph, ["pos"])
        k = TorchUtils.validateKNNEdgeIndex(edge_index)
        ei = _nat.i64(edge_index)
        order = torch.argsort(ei[0], stable=True)          # group rows by centre, as edge_index[0].view(-1, k)
        nbr = ei[1][order].contiguous()
        _, eigvec = _nat.pca_dense(_nat.f32(_graph.pos), nbr, k)
        return eigvec.to(_graph.pos.device)

    def calculateEdgeCost(self) -> None:
        """edge_attr = 1 - |n_i · n_j| (GraphBuilder.py:134-145)."""
        _graph = self.graph
        GeneralUtils.validateAttributes(_graph, ["edge_index", "n"])
        normals = _graph.n[_graph.edge_index]
        _graph.edge_attr = 1 - (normals[0] * normals[1]).sum(dim=-1).abs_()

    def flipNormals(self) -> None:
        """MST over 1-|n_i·n_j| then sign propagation from the highest point (GraphBuilder.py:129-209), on the GPU."""
        _graph = self.graph
        GeneralUtils.validateAttributes(_graph, ["pos", "n", "edge_index"])
        ei = _graph.edge_index.detach()
        n = _nat.orient_normals_mst_gpu(_graph.pos.detach(), _graph.n.detach(), ei[0], ei[1])
        _graph.n = n.to(device=_graph.pos.device, dtype=_graph.pos.dtype)
