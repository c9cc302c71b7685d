#!/usr/bin/env python
"""ResNet-50 downsample 1x1 convolutions (batch 256, bf16 NHWC): our GEMM with the stride-2 row
gather and the BatchNorm statistics epilogue vs MIOpen's forward + the separate statistics pass.

usage: python scripts/bench_ds.py [batch] [engine ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops.gemm import SHARDS, gemm  # noqa: E402
from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE  # noqa: E402
from fluxmpi_amd.utils.miopen import install_tuned_db  # noqa: E402


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
    install_tuned_db()
    torch.backends.cudnn.benchmark = True
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    engines = [int(e) for e in sys.argv[2:]] or [2]
    C = _ext.get(required=True)
    for H, ci, co, s in ((56, 64, 256, 1), (56, 256, 512, 2), (28, 512, 1024, 2), (14, 1024, 2048, 2)):
        x = torch.randn(B, ci, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device="cuda") * 0.05).to(torch.bfloat16)
        ho = (H + s - 1) // s
        M = B * ho * ho
        c = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
        stats = torch.zeros(SHARDS * 2 * co, device="cuda")
        x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
        w2 = w.view(co, ci)
        r = {"H": H, "ci": ci, "co": co, "stride": s}
        for eng in engines:
            r[f"ours_e{eng}"] = round(bench(lambda: gemm(x2, w2, c, M=M, N=co, K=ci, lda=ci, ldb=ci, ldc=co, mode=1,
                                                         stats=stats, a_sub=(H, H) if s == 2 else None,
                                                         engine=eng)), 1)
        y = torch.nn.functional.conv2d(x, w, None, s)
        r["miopen"] = round(bench(lambda: torch.nn.functional.conv2d(x, w, None, s)), 1)
        f = [torch.ones(co, device="cuda") for _ in range(4)]  # weight, bias, mean, invstd
        r["stats_pass"] = round(bench(lambda: C.bn_stats_finalize(
            y.data_ptr(), f[0].data_ptr(), f[1].data_ptr(), 0, 0, f[2].data_ptr(), f[3].data_ptr(), 0, 0,
            stats.data_ptr(), M, co, 0.1, 1e-5, 0, DTYPE_CODE[torch.bfloat16], torch.cuda.current_stream().cuda_stream,
            0)), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
