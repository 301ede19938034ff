"""Noise synthesis (drop-in for Pointcloud/Modules/Noise.py:24-88).

σ = mean_edge_length · level; Gaussian offset along the normal (direction 0) or isotropic (direction 1);
impulsive noise keeps only a `level` fraction of the offsets.  Uses torch's RNG on the graph's device
(optionally a caller generator for reproducible fixtures).
"""
from __future__ import annotations

import torch


class Noise:

    def __init__(self, graph):
        self.graph = graph
        self.noise_level = None
        self.noise_type = None
        self.noise_direction = None

    def generateNoise(self, noise_level, mean_edge_length, noise_type: int = 0, noise_direction: int = 0,
                      keepNormals: bool = False, generator: torch.Generator = None):
        in_range = lambda x, start, end: (x - (end - start) * 0.5) ** 2
        if in_range(noise_level, 0, 1) > in_range(0, 0, 1):
            raise ValueError(f"noise_level is {noise_level}, but should be a positive number!")
        if in_range(noise_type, 0, 1) > in_range(0, 0, 1):
            raise ValueError(f"noise_type is {noise_type}, but should be a number between 0 and 1!")
        if in_range(noise_direction, 0, 1) > in_range(0, 0, 1):
            raise ValueError(f"noise_direction is {noise_direction}, but should be a number between 0 and 1!")
        self.noise_level, self.noise_type, self.noise_direction = noise_level, noise_type, noise_direction
        gt, _ = self.getGT()
        n = self.graph.num_nodes
        std = float(mean_edge_length) * noise_level
        r = torch.randn((n, 3), generator=generator, device=gt.device if generator is None else generator.device,
                        dtype=torch.float32).to(gt.device) * std
        offset = r if noise_direction == 1 else self.graph.n * r[:, 0, None]
        if noise_type == 1:
            # the reference draws torch_randperm(n) on the CPU default generator (Noise.py:56); a caller generator
            # draws on its own device
            gdev = "cpu" if generator is None else generator.device
            drop = torch.randperm(n, generator=generator, device=gdev)[:int(n * (1 - noise_level))].to(gt.device)
            offset[drop] = 0
        self.setNoise(gt + offset, keepNormals)

    def getGT(self):
        g = self.graph
        pos = g.gt if hasattr(g, "gt") else g.pos
        nrm = g.gt_n if hasattr(g, "gt_n") else g.n
        return pos, nrm

    def setNoise(self, noise: torch.Tensor, keepNormals: bool = False):
        g = self.graph
        g.gt, g.gt_n = self.getGT()
        g.pos = noise
        if not keepNormals:
            delattr(g, "n")

    def resetNoise(self):
        g = self.graph
        if not hasattr(g, "gt"):
            raise ValueError("Can't reset noise if noise has never been applied")
        g.pos = g.gt
        self.noise_level = self.noise_type = self.noise_direction = None
