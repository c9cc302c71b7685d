#!/usr/bin/env python
"""Fused NHWC GroupNorm forward / backward (groupnorm.hip) at the DEQ cells' shapes: us per call and
the algorithmic TB/s (each tensor read / written once). FLUXMPI_C_VARIANT=<.so> (through
scripts/diag/load_variant.py) times a variant build. JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
import load_variant  # noqa: E402

load_variant.install()
import torch  # noqa: E402
from fluxmpi_amd.ops.groupnorm import gn_bwd_raw, gn_fwd_raw  # noqa: E402


def t_us(fn, iters=20, repeats=3):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(repeats):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    torch.manual_seed(0)
    cl = torch.channels_last
    for (n, c, h, w, g) in [(256, 512, 16, 16, 16), (256, 48, 28, 28, 8), (256, 128, 32, 32, 16)]:
        x = torch.randn(n, c, h, w, device="cuda").bfloat16().contiguous(memory_format=cl)
        a = torch.randn_like(x)
        wt, b = torch.randn(c, device="cuda"), torch.randn(c, device="cuda")
        y, hsv, mean, rstd, w32 = gn_fwd_raw(x, a, wt, b, g, 1e-5, True)
        dy = torch.randn_like(x)
        fwd = t_us(lambda: gn_fwd_raw(x, a, wt, b, g, 1e-5, True))
        bwd = t_us(lambda: gn_bwd_raw(dy, hsv, mean, rstd, w32, g, True))
        byt = x.numel() * 2
        print(json.dumps({"shape": [n, c, h, w], "groups": g, "variant": os.environ.get("FLUXMPI_C_VARIANT", ""),
                          "fwd_add_relu_us": round(fwd, 1), "fwd_tbs": round(4 * byt / fwd / 1e6, 2),
                          "bwd_relu_us": round(bwd, 1), "bwd_tbs": round(3 * byt / bwd / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
