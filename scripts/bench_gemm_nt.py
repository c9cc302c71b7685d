#!/usr/bin/env python
"""gemm_nt.hip (ping-pong 8-wave 256x256 NT GEMM) vs hipBLASLt (torch), TFLOP/s on
uniform [-1, 1) bf16 operands (cdna_hip_programming.md rule 25), interleaved rounds in one process.

Split-K tail arms: nt_s<k> = the default kernel with FLUXMPI_GEMM_NT_SPLIT = k (0: off, the default; nt = the current setting).

Shapes: 4096^3 and the ViT-B/16 Linears at batch 256 (M = 50432 tokens), forward (x W^T),
input gradient (dy W, ours on W^T), fc1 forward + bias + GELU (EPI 1), fc2 input gradient +
GELU backward + bias-gradient partials (EPI 2). Every kernel is checked against an fp32 torch
matmul of the same bf16 operands before it is timed.

usage: python scripts/bench_gemm_nt.py [--quick]  -> JSON lines
"""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import _ext  # noqa: E402


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


def uni(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).bfloat16()


def check(name, got, ref, tol=2e-2):
    err = ((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
    ok = err < tol
    print(json.dumps({"check": name, "rel_max_err": round(err, 6), "ok": ok}), flush=True)
    if not ok:
        raise SystemExit(f"{name}: wrong result (rel max err {err})")


def checks_only(C, st, name, m, n, k):
    a = uni(m, k)
    w = (uni(n, k) * (k ** -0.5)).bfloat16()
    bias = (torch.rand(n, device="cuda") - 0.5).float()
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    c2 = torch.empty_like(c)
    ref = a.float() @ w.float().t()
    for bdt in (torch.float32, torch.bfloat16):
        b = bias.to(bdt)
        for _ in range(2):
            C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), 0, b.data_ptr(), int(bdt == torch.float32), 0, 0,
                      k, k, n, m, n, k, 0, st)
            torch.cuda.synchronize()
            check(f"{name}_epi0_bias_{str(bdt)[6:]}", c, ref + b.float())
    C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), c2.data_ptr(), bias.data_ptr(), 1, 0, 0,
              k, k, n, m, n, k, 1, st)
    torch.cuda.synchronize()
    check(f"{name}_epi1_g", c2, torch.nn.functional.gelu((ref + bias).bfloat16().float(), approximate="tanh"))


SPLITS = tuple(int(v) for v in os.environ.get("BENCH_NT_SPLITS", "0,8,16,24,32").split(","))


def main():
    C = _ext.get(required=True)
    st = torch.cuda.current_stream().cuda_stream
    quick = "--quick" in sys.argv
    shapes = [("sq4096", 4096, 4096, 4096)]
    M = 50432
    shapes += [("qkv", M, 2304, 768), ("proj", M, 768, 768), ("fc1", M, 3072, 768), ("fc2", M, 768, 3072),
               ("qkv_dgrad", M, 768, 2304), ("fc1_dgrad", M, 768, 3072), ("fc2_dgrad", M, 3072, 768)]
    if quick:
        shapes = shapes[:3]
    # correctness-only shapes: odd k-tile counts (LDS buffer parity flips between tiles), the
    # minimum K, ranges of a few units, one tile split over 128 workgroups (127 contributors)
    for name, m, n, k in (("odd_nk13", 256 * 41, 768, 832), ("nk2", 256 * 37, 512, 128), ("nk3", 256 * 300, 256, 192),
                          ("one_tile", 256, 256, 8192), ("few_tiles", 512, 768, 4096), ("u_lt_g", 256, 512, 1344)):
        checks_only(C, st, name, m, n, k)
    for name, m, n, k in shapes:
        a = uni(m, k)
        w = uni(n, k) * (k ** -0.5)
        w = w.bfloat16()
        bias = (torch.rand(n, device="cuda") - 0.5).float()
        c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        c2 = torch.empty_like(c)
        fl = 2.0 * m * n * k

        def ours(epi=0, h=None, part=None, bias_=None):
            C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), c2.data_ptr() if epi == 1 else 0,
                      bias_.data_ptr() if bias_ is not None else 0, 1, h.data_ptr() if h is not None else 0,
                      part.data_ptr() if part is not None else 0, k, k, n, m, n, k,
                      epi, st)

        ref = a.float() @ w.float().t()
        ours()
        torch.cuda.synchronize()
        check(f"{name}_epi0", c, ref)
        ours(0, bias_=bias)
        check(f"{name}_epi0_bias", c, ref + bias)
        def dgelu(hf):
            t = torch.tanh(0.7978845608 * (hf + 0.044715 * hf ** 3))
            return 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * 0.7978845608 * (1 + 3 * 0.044715 * hf * hf)

        ours(1, bias_=bias)
        hb = (ref + bias).bfloat16()
        check(f"{name}_epi1_dgelu", c, dgelu(hb.float()))  # EPI 1 stores gelu'(h), not h
        check(f"{name}_epi1_g", c2, torch.nn.functional.gelu(hb.float(), approximate="tanh"))
        h = uni(m, n)
        dgel = dgelu(h.float())
        h = dgel.bfloat16()  # EPI 2 reads the derivative as EPI 1 stored it
        part = torch.empty(C.gemm_nt_colpart_rows(m), n, device="cuda", dtype=torch.float32)
        ours(2, h=h, part=part)
        dh_ref = ref.bfloat16().float() * dgel
        check(f"{name}_epi2_dh", c, dh_ref)
        check(f"{name}_epi2_db", part.sum(0), dh_ref.sum(0), tol=5e-2)
        del ref, dh_ref, dgel

        best: dict = {}
        wt = w.t().contiguous()  # the [K][N] layout hipBLASLt's dgrad form reads (dy @ W)
        for rnd in range(3):
            best.setdefault("blas", []).append(t_us(lambda: torch.matmul(a, wt)))
            best.setdefault("blas_bias", []).append(t_us(lambda: torch.nn.functional.linear(a, w, bias.bfloat16())))
            for sm in SPLITS:  # the split-K tail's minimum share (0: the last round tile-granular)
                C.gemm_nt_set_split(sm)
                best.setdefault(f"nt_s{sm}", []).append(t_us(lambda: ours()))
                best.setdefault(f"nt_epi2_s{sm}", []).append(t_us(lambda: ours(2, h=h, part=part)))
            C.gemm_nt_set_split(0)
            best.setdefault("nt", []).append(t_us(lambda: ours()))
            best.setdefault("nt_bias", []).append(t_us(lambda: ours(0, bias_=bias)))
            best.setdefault("nt_gelu", []).append(t_us(lambda: ours(1, bias_=bias)))
            best.setdefault("nt_epi2", []).append(t_us(lambda: ours(2, h=h, part=part)))
        rec = {"shape": name, "M": m, "N": n, "K": k}
        for key, v in best.items():
            us = min(v)
            rec[key + "_us"] = round(us, 1)
            rec[key + "_tfs"] = round(fl / us / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del a, w, c, c2, h, part, wt
        torch.cuda.empty_cache()
    # the W^T transpose the input-gradient path runs per call
    for r, cc in ((768, 3072), (3072, 768), (2304, 768)):
        src = uni(r, cc)
        dst = torch.empty(cc, r, device="cuda", dtype=torch.bfloat16)
        C.transpose_bf16(src.data_ptr(), dst.data_ptr(), r, cc, cc, r, st)
        torch.cuda.synchronize()
        assert torch.equal(dst, src.t()), "transpose_bf16 mismatch"
        us = t_us(lambda: C.transpose_bf16(src.data_ptr(), dst.data_ptr(), r, cc, cc, r, st))
        print(json.dumps({"transpose": [r, cc], "us": round(us, 2), "TBs": round(4 * r * cc / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
