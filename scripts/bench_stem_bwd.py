#!/usr/bin/env python
"""Stem backward kernel time (ResNet-50 stem, batch 256) from a rocprof-free event timing of the
fused stem's forward + backward minus its forward. Run once per FLUXMPI_STEM_BWD_DIAG mode
(0 normal, 1 no MFMA phase, 2 no pool-gradient gather, 3 no next-iteration loads) to split the
kernel's time between its phases; the diagnostic modes produce wrong gradients by design."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from fluxmpi_amd.models import resnet as R
    from fluxmpi_amd.ops import stem as S
    B = int(os.environ.get("B", 256))
    x3 = torch.randn(B, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda()
    bn = R._norm(64, "fused").cuda()
    y = S.stem(x3, conv, bn)
    gy = torch.randn_like(y)
    fwd = bench(lambda: S.stem(x3, conv, bn))
    both = bench(lambda: S.stem(x3, conv, bn).backward(gy))
    print(json.dumps({"bench": "stem_bwd", "mode": int(os.environ.get("FLUXMPI_STEM_BWD_DIAG", "0")),
                      "batch": B, "fwd_us": round(fwd, 1), "fwd_bwd_us": round(both, 1),
                      "bwd_us": round(both - fwd, 1)}), flush=True)


if __name__ == "__main__":
    main()
