"""The README quick-start model (reference ``README.md:37-38``):

    Chain(Dense(1 => 256, tanh), Dense(256 => 512, tanh), Dense(512 => 256, tanh), Dense(256 => 1))

263,681 parameters in 8 leaves.
"""
from __future__ import annotations

import torch.nn as nn

README_MLP = (1, 256, 512, 256, 1)


def mlp(sizes=README_MLP) -> nn.Sequential:
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers.append(nn.Tanh())
    return nn.Sequential(*layers)
