#!/usr/bin/env python
"""Print the per-shape kernel choices the hybrid ResNet-50 makes at its first step (our kernels
vs MIOpen: 1x1 forwards, 3x3 forwards, weight gradients), after two bench-config steps."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.models import resnet50  # noqa: E402
from fluxmpi_amd.ops import fused_block as fb  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402


def main():
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    model = resnet50(num_classes=1000, conv_impl="hybrid", norm="fused").to(dev, memory_format=torch.channels_last)
    for m in model.modules():
        if not isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    x = torch.randn(256, 3, 224, 224, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (256,), device=dev)
    for _ in range(2):
        F.cross_entropy(model(x).float(), y).backward()
    torch.cuda.synchronize()
    for line in fb.dump_choices():  # the format fb.load_choices / bench.py --choices read
        print(line)


if __name__ == "__main__":
    main()
