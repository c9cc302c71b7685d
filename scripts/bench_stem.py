#!/usr/bin/env python
"""ResNet-50 stem (7x7/2, 64 filters, 224x224, batch 256, bf16 NHWC).

1. MIOpen with the input channels padded 3 -> 4 / 8 (zero channel, zero weights: same math):
   forward, weight gradient, and the pad copy itself.
2. The whole stem (conv -> BN -> ReLU -> max-pool), forward and forward + backward: the MFMA
   stem kernels (ops/stem.py) vs the padded MIOpen conv + ops/pool.py's fused BN/ReLU/pool."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    x3 = torch.randn(B, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    for cin in (3, 4, 8):
        x = F.pad(x3, (0, 0, 0, 0, 0, cin - 3)).contiguous(memory_format=torch.channels_last) if cin > 3 else x3
        w = (torch.randn(64, cin, 7, 7, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=2, padding=3)
        dy = torch.randn_like(y)
        rec = {"cin": cin,
               "fwd_us": bench(lambda: F.conv2d(x, w, stride=2, padding=3)),
               "wgrad_us": bench(lambda: torch.ops.aten.convolution_backward(
                   dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))}
        if cin > 3:
            rec["pad_us"] = bench(lambda: F.pad(x3, (0, 0, 0, 0, 0, cin - 3)).contiguous(
                memory_format=torch.channels_last))
        print(json.dumps(rec), flush=True)

    from fluxmpi_amd.models import resnet as R
    from fluxmpi_amd.ops import pool
    from fluxmpi_amd.ops import stem as S
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda()
    bn = R._norm(64, "fused").cuda()
    w4 = torch.nn.functional.pad(conv.weight.detach(), (0, 0, 0, 0, 0, 1)).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_(True)

    def old_fwd():
        return pool.bn_relu_maxpool(F.conv2d(pool.pad_c3_to_c4(x3), w4, None, 2, 3), bn, 3, 2, 1)

    def new_fwd():
        return S.stem(x3, conv, bn)

    y = new_fwd()
    gy = torch.randn_like(y)
    rec = {"stem": "fused", "ours_fwd_us": bench(new_fwd), "miopen_fwd_us": bench(old_fwd),
           "ours_fwd_bwd_us": bench(lambda: new_fwd().backward(gy)),
           "miopen_fwd_bwd_us": bench(lambda: old_fwd().backward(gy))}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
