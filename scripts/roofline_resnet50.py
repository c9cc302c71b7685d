#!/usr/bin/env python
"""Roofline table of ResNet-50's convolution and BatchNorm kernels at the bench config (batch 256,
bf16 NHWC): for every distinct (op, shape) — achieved TFLOP/s and TB/s of our kernel and of
MIOpen, against MI355X's dense bf16 peak (2.5 PF/s) and HBM peak (8 TB/s spec, ~6.3 measured).

Bytes are the minimum traffic (each operand read once, the output written once; split-K partials
and L2 re-reads not counted), so TB/s is an "algorithmic" rate. Each row's `calls` is how many
times the op runs per training step; `chosen` marks the faster implementation (the model picks
per shape the same way, measured once at the first step).

usage: python scripts/roofline_resnet50.py [out.md]   (prints markdown; JSON lines to stderr)
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import gemm as G  # noqa: E402
from fluxmpi_amd.ops.batchnorm import fused_batch_norm  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402

PEAK_TF = 2500.0
PEAK_TBS = 8.0


def t_us(fn, iters=10, repeats=3):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(repeats):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def t_us_graph(fn, iters=10, repeats=3):
    """``t_us`` over a HIP-graph replay of ``iters`` calls of ``fn``: the GPU time of its kernels
    back to back, without the host's autograd / launch cost between them (an eager loop of a
    ~25 us BatchNorm backward through autograd.grad is host-bound: it measured 131-160 us for
    every shape)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    return t_us(g.replay, iters=1, repeats=repeats) / iters


def conv_ops(B=256):
    """(kind, H_in, cin, cout, stride) -> calls per step, for torchvision-v1.5 ResNet-50."""
    ops: dict = {}

    def add(k):
        ops[k] = ops.get(k, 0) + 1

    h_prev, cin0 = 56, 64
    for hout, mid, out, nb, stride in [(56, 64, 256, 3, 1), (28, 128, 512, 4, 2), (14, 256, 1024, 6, 2),
                                       (7, 512, 2048, 3, 2)]:
        for b in range(nb):
            cin = cin0 if b == 0 else out
            hin = h_prev if b == 0 else hout
            s = stride if b == 0 else 1
            add(("1x1", hin, cin, mid, 1))
            add(("3x3", hin, mid, mid, s))
            add(("1x1", hout, mid, out, 1))
            if b == 0:
                add(("1x1", hin, cin, out, s))
        h_prev, cin0 = hout, out
    return ops


def bench_conv(kind, hin, cin, cout, s, B):
    dev = "cuda"
    ho = (hin + s - 1) // s if kind == "1x1" else (hin + 1) // 2 if s == 2 else hin
    x = torch.randn(B, cin, hin, hin, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    k = 1 if kind == "1x1" else 3
    w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, cout, ho, ho, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    pad = 1 if kind == "3x3" else 0
    M_out = B * ho * ho
    kk = cin * k * k
    flops = 2.0 * M_out * cout * kk
    bx, by, bw = x.numel() * 2, dy.numel() * 2, w.numel() * 2
    stats = torch.zeros(64, 2, cout, device=dev)
    res = {}
    # forward
    res["fwd_miopen"] = t_us(lambda: F.conv2d(x, w, None, s, pad))
    if kind == "1x1" and s == 1:
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        res["fwd_ours"] = t_us(lambda: G.conv1x1_fwd(x2, w.view(cout, cin), None, stats))
    elif kind == "3x3" and s == 1:
        res["fwd_ours"] = t_us(lambda: G.conv3x3_fwd(x, w, stats=stats))
    elif kind == "3x3" and s == 2:
        res["fwd_ours"] = t_us(lambda: G.conv3x3_s2_fwd(x, w, stats=stats))
    # input gradient
    xe = torch.empty_like(x)
    res["dgrad_miopen"] = t_us(lambda: torch.ops.aten.convolution_backward(
        dy, xe, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False]))
    if kind == "1x1" and s == 1:
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        G.note_filter(w)
        res["dgrad_ours"] = t_us(lambda: G.conv1x1_dgrad(dy2, w.view(cout, cin), w4d=w))
    elif kind == "3x3" and s == 1:
        G.note_filter(w)
        res["dgrad_ours"] = t_us(lambda: G.conv3x3_dgrad(dy, w))
    # weight gradient
    res["wgrad_miopen"] = t_us(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False]))
    if kind == "1x1" and s == 1:
        res["wgrad_ours"] = t_us(lambda: G.conv1x1_wgrad_v2(dy.permute(0, 2, 3, 1).reshape(-1, cout),
                                                            x.permute(0, 2, 3, 1).reshape(-1, cin)))
    elif kind == "1x1" and s == 2:
        res["wgrad_ours"] = t_us(lambda: G.conv1x1_wgrad_s2(dy.permute(0, 2, 3, 1).reshape(-1, cout), x))
    elif kind == "3x3" and s == 1:
        res["wgrad_ours"] = t_us(lambda: G.conv3x3_wgrad(dy, x))
    else:
        res["wgrad_ours"] = t_us(lambda: G.conv3x3_wgrad_s2(dy, x))
    out = []
    for op, byts in (("fwd", bx + bw + by), ("dgrad", by + bw + bx), ("wgrad", by + bx + bw)):
        cand = {impl: res[f"{op}_{impl}"] for impl in ("ours", "miopen") if f"{op}_{impl}" in res}
        chosen = min(cand, key=cand.get)
        for impl, us in cand.items():
            out.append({"op": f"{kind}/s{s} {op}", "shape": f"{B}x{hin}x{hin}x{cin}->{cout}", "impl": impl,
                        "chosen": impl == chosen, "us": round(us, 1), "gflop": round(flops / 1e9, 1),
                        "mbytes": round(byts / 1e6, 1), "tflops": round(flops / us / 1e6, 1),
                        "tbs": round(byts / us / 1e6, 2)})
    return out


def bench_bn(c, h, relu, res, B):
    """The BatchNorm forward / backward as the model runs them (the fused kernels through their raw
    bindings, the calls ``ops/batchnorm._FusedBN`` makes), timed by graph replay: no autograd,
    no host launch cost between the kernels (an eager autograd.grad loop was host-bound at
    131-160 us for every shape; capturing autograd itself crashed)."""
    from fluxmpi_amd.ops import _ext
    from fluxmpi_amd.ops.batchnorm import _workspace
    from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE
    C = _ext.get(required=True)
    x = torch.randn(B, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    rows = x.numel() // c
    w32, b32 = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    y, dy, dx = torch.empty_like(x), torch.randn_like(x), torch.empty_like(x)
    dres = torch.empty_like(x) if res else None
    mean, inv = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    dw, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    mask = torch.empty(x.numel() // 8, device="cuda", dtype=torch.uint8) if (relu and res) else None
    ws = _workspace(x)
    code = DTYPE_CODE[x.dtype]

    def s():
        return torch.cuda.current_stream().cuda_stream

    def fwd():
        C.bn_fwd_train(x.data_ptr(), y.data_ptr(), r.data_ptr() if r is not None else 0, w32.data_ptr(), b32.data_ptr(),
                       rm.data_ptr(), rv.data_ptr(), mean.data_ptr(), inv.data_ptr(), ws.data_ptr(), rows, c, 0.1,
                       1e-5, int(relu), mask.data_ptr() if mask is not None else 0, code, s(), 0)

    def bwd():
        C.bn_bwd(dy.data_ptr(), x.data_ptr(), 0, mask.data_ptr() if mask is not None else 0, w32.data_ptr(),
                 b32.data_ptr(), mean.data_ptr(), inv.data_ptr(), dx.data_ptr(),
                 dres.data_ptr() if dres is not None else 0, dw.data_ptr(), db.data_ptr(), ws.data_ptr(), rows, c,
                 int(relu), code, s(), 0)

    fwd()
    torch.cuda.synchronize()
    fwd_us = t_us_graph(fwd)
    bwd_us = t_us_graph(bwd)
    n = x.numel()
    return [{"op": f"bn{'+res' if res else ''}{'+relu' if relu else ''} fwd", "shape": f"{B}x{h}x{h}x{c}",
             "impl": "ours", "chosen": True, "us": round(fwd_us, 1), "gflop": 0.0,
             "mbytes": round((2 * n * 2 + (n * 2 if res else 0)) / 1e6, 1),
             "tflops": 0.0, "tbs": round((2 * n * 2 + (n * 2 if res else 0)) / fwd_us / 1e6, 2)},
            {"op": f"bn{'+res' if res else ''}{'+relu' if relu else ''} bwd", "shape": f"{B}x{h}x{h}x{c}",
             "impl": "ours", "chosen": True, "us": round(bwd_us, 1), "gflop": 0.0,
             "mbytes": round((3 * n * 2 + (n * 2 if res else 0)) / 1e6, 1), "tflops": 0.0,
             "tbs": round((3 * n * 2 + (n * 2 if res else 0)) / bwd_us / 1e6, 2)}]


def main():
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    B = 256
    rows = []
    ops = conv_ops(B) if not os.environ.get("ROOFLINE_BN_ONLY") else {}
    for (kind, hin, cin, cout, s), calls in ops.items():
        for r in bench_conv(kind, hin, cin, cout, s, B):
            r["calls"] = calls
            rows.append(r)
            print(json.dumps(r), file=sys.stderr, flush=True)
    for c, h, relu, res, calls in [(64, 56, True, False, 6), (256, 56, True, True, 3), (128, 28, True, False, 8),
                                   (512, 28, True, True, 4), (256, 14, True, False, 12), (1024, 14, True, True, 6),
                                   (512, 7, True, False, 6), (2048, 7, True, True, 3)]:
        for r in bench_bn(c, h, relu, res, B):
            r["calls"] = calls
            rows.append(r)
            print(json.dumps(r), file=sys.stderr, flush=True)
    lines = ["| op | shape (N x H x W x C -> Cout) | calls/step | impl | us | TFLOP/s | % of 2.5 PF | TB/s (min bytes) "
             "| % of 8 TB/s |", "|---|---|---|---|---|---|---|---|---|"]
    tot_chosen = 0.0
    for r in rows:
        mark = "**" if r["chosen"] else ""
        lines.append(f"| {r['op']} | {r['shape']} | {r['calls']} | {mark}{r['impl']}{mark} | {r['us']} | {r['tflops']} | "
                     f"{100 * r['tflops'] / PEAK_TF:.0f} | {r['tbs']} | {100 * r['tbs'] / PEAK_TBS:.0f} |")
        if r["chosen"]:
            tot_chosen += r["us"] * r["calls"]
    lines.append("")
    lines.append(f"Sum over ops of the faster implementation x calls/step: {tot_chosen / 1e3:.2f} ms/step "
                 "(isolated, L2-cold between ops differs from the in-model profile).")
    md = "\n".join(lines)
    print(md)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(md + "\n")


if __name__ == "__main__":
    main()
