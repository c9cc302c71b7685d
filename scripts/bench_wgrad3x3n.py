#!/usr/bin/env python
"""wgrad3x3n.hip (narrow-channel 3x3 weight gradient, input rows staged once per 4-row block) in each
autotune configuration vs the split-K im2col kernel (gemm_wgrad, best of its autotune configs) vs
MIOpen, at the ResNet-50 stage-1 / stage-2 shapes (batch 256). Times include the split-K reduce.
Interleaved rounds, best of 3, us and TFLOP/s -> JSON lines. Checked against the im2col kernel first."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import conv_choice as CC  # noqa: E402
from fluxmpi_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    torch.backends.cudnn.benchmark = True
    for (n, c, h, w) in [(256, 64, 56, 56), (256, 128, 28, 28)]:
        x = (torch.rand(n, c, h, w, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = (torch.rand(n, c, h, w, device="cuda") * 2 - 1).bfloat16().contiguous(memory_format=torch.channels_last)
        wt = torch.zeros(c, c, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = G.conv3x3_wgrad(dy, x).float()
        errs = {}
        for cfg in CC.w3n_configs(c):
            d = G.conv3x3_wgrad_n(dy, x, *cfg).float()
            errs[str(cfg)] = round(float((d - ref).norm() / ref.norm()), 5)
            assert errs[str(cfg)] < 5e-3, errs
        fl = 2.0 * n * h * w * c * 9 * c
        arms = {f"w3n_{v}_{t}": (lambda v=v, t=t: G.conv3x3_wgrad_n(dy, x, v, t)) for v, t in CC.w3n_configs(c)}
        for v, t in CC._WG_CONFIGS:
            arms[f"im2col_{v}_{t}"] = lambda v=v, t=t: CC._with_cfg((v, t), lambda: G.conv3x3_wgrad(dy, x))
        arms["miopen"] = lambda: torch.ops.aten.convolution_backward(dy, x, wt, None, [1, 1], [1, 1], [1, 1], False,
                                                                     [0, 0], 1, [False, True, False])[1]
        best: dict = {}
        for _ in range(3):
            for k, f in arms.items():
                best.setdefault(k, []).append(t_us(f))
        rec = {"shape": [n, c, h, w], "check_rel": errs}
        for k, v in best.items():
            rec[k + "_us"] = round(min(v), 1)
        for pre in ("w3n", "im2col"):
            k = min((k for k in best if k.startswith(pre)), key=lambda k: min(best[k]))
            rec[pre + "_best"] = k
            rec[pre + "_best_tfs"] = round(fl / min(best[k]) / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
