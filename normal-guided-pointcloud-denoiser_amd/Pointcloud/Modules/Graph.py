"""Attribute bag standing in for torch_geometric.data.Data as the reference's shared `graph` object.

Only what the hot path reads: pos, n, edge_index, edge_attr, gt, gt_n; num_nodes = pos.size(0),
num_edges = edge_index.size(1) (GraphBuilder.py:50 creates it, every helper shares it).
"""
from __future__ import annotations


class Data:
    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        return self.pos.size(0)

    @property
    def num_edges(self) -> int:
        return self.edge_index.size(1)

    def __repr__(self):
        items = ", ".join(f"{k}={list(v.shape) if hasattr(v, 'shape') else v}" for k, v in vars(self).items())
        return f"Data({items})"
