"""Model zoo for the benchmark configs (BASELINE.json):

* ``mlp``       — the README 4-layer Dense MLP (reference ``README.md:37-38``)
* ``resnet50``  — ResNet-50 (Lux ImageNet example; the headline benchmark)
* ``vit_b16``   — ViT-Base/16
* ``deq``       — a Deep Equilibrium Model (FastDEQ-style implicit layer, MNIST-shaped, 48 channels)
* ``deq_cifar`` — the FastDEQ-width DEQ (CIFAR-shaped, 512 channels, 10.6 MB of bf16 gradients)
"""
from __future__ import annotations

from .mlp import README_MLP, mlp  # noqa: F401
from .resnet import ResNet, resnet18ish, resnet50  # noqa: F401


def build_model(name: str, **kw):
    name = name.lower()
    if name == "resnet50":
        return resnet50(**kw)
    if name in ("resnet_tiny", "resnet18ish"):
        return resnet18ish(**kw)
    if name == "mlp":
        return mlp()
    if name in ("vit_b16", "vit"):
        from .vit import vit_b16
        kw.pop("conv_impl", None)
        kw.pop("norm", None)
        return vit_b16(**kw)
    if name == "deq":
        from .deq import deq_mnist
        kw.pop("conv_impl", None)
        kw.pop("norm", None)
        return deq_mnist(**kw)
    if name == "deq_cifar":
        from .deq import deq_cifar
        kw.pop("conv_impl", None)
        kw.pop("norm", None)
        return deq_cifar(**kw)
    raise ValueError(f"unknown model {name!r}")
