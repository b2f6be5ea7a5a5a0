"""MNIST-style MLP (north-star config #1: "local provider single-node, AI runtime MNIST MLP
on CPU"; reference examples/runtime/ai/basics/**/mnist-*.py) plus a synthetic MNIST-shaped
dataset (no downloads: class-conditional 28x28 patterns with noise, learnable to ~100%).

On GPU the layers use cloudtik_amd.ops.linear (weight-gradient GEMM accumulating into the
flat gradient buffer); on CPU plain torch.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, in_features: int = 784, hidden: Sequence[int] = (512, 256), num_classes: int = 10,
                 dropout: float = 0.0, device=None, dtype=torch.float32):
        super().__init__()
        dims = [in_features] + list(hidden) + [num_classes]
        self.layers = nn.ModuleList(nn.Linear(a, b, device=device, dtype=dtype) for a, b in zip(dims[:-1], dims[1:]))
        self.dropout = dropout

    def forward(self, x):
        from cloudtik_amd import ops
        x = x.reshape(x.shape[0], -1).to(self.layers[0].weight.dtype)
        for i, layer in enumerate(self.layers):
            x = ops.linear(x, layer.weight, layer.bias)
            if i < len(self.layers) - 1:
                x = torch.relu(x)
                if self.dropout and self.training:
                    x = nn.functional.dropout(x, self.dropout)
        return x


def synthetic_mnist(n: int, seed: int = 0, noise: float = 1.5) -> Tuple[torch.Tensor, torch.Tensor]:
    """[n, 1, 28, 28] float images in [0, 1] and int64 labels; class c is a fixed random
    stroke pattern plus noise, so a model can learn it but not memorise a single image."""
    g = torch.Generator().manual_seed(1234)       # class templates: identical on every rank
    templates = (torch.rand(10, 28, 28, generator=g) > 0.75).float()
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    x = templates[y] * (0.6 + 0.4 * torch.rand(n, 1, 1, generator=g)) + noise * torch.rand(n, 28, 28, generator=g)
    return x.clamp(0, 1).unsqueeze(1), y
