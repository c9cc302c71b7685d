"""``nn.Linear`` for token-major activations with MI355X-shaped GEMMs.

Forward and input gradient run on ``gemm_nt.hip`` (persistent ping-pong 256x256 MFMA tiles,
bias in the epilogue; ``ops/gemm_nt.py``) when the token count and widths tile exactly
(ViT-B/16: 50432 = 197 x 256 tokens), else hipBLASLt (``F.linear``, ``dy @ W``). The weight gradient ``dW = dY^T X`` is the awkward one:
K = tokens (50432 for ViT-B/16 at batch 256) and a small output (768..3072 squared), so
hipBLASLt's 256x256 tiles leave most of the 256 CUs idle (36-108 workgroups; 312-431 us
per call, ``profiles/r1_vit_b16_s61_steady.md``). It runs on our split-K MFMA kernels
instead: ``wgrad256.hip`` (256x256 tiles, 8 waves, 4-stage LDS-DMA ring, transposed LDS
reads; 0.91-0.98 PF/s on the ViT shapes) when both widths are multiples of 256, else
``gemm_glds.hip``'s 128x128 kernel; fp32 partials + one reduce, split counts measured by
``scripts/bench_vit_gemm.py``. The bias gradient is the
``colsum`` HIP kernel (one read of dy at HBM rate) instead of autograd's generic reduction.

``WGRAD_MODE = "torch"`` keeps hipBLASLt for the weight gradient (A/B runs).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext
from . import graddst
from .multi_tensor import DTYPE_CODE

# (N_out, N_in) -> split-K factor, from scripts/bench_vit_gemm.py on MI355X (M = 50432 tokens)
_SPLITS = {(2304, 768): 16, (768, 768): 16, (3072, 768): 8, (768, 3072): 4}


# "ours": the split-K 256x256 weight-gradient kernel where it applies; "torch": hipBLASLt (A/B, tests)
WGRAD_MODE = "ours"


def _wgrad_mode() -> str:
    return WGRAD_MODE


def native_ok(x2: torch.Tensor, dy2: torch.Tensor) -> bool:
    """Shapes / layouts the HIP weight-gradient and column-sum kernels take."""
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16 and x2.is_contiguous()
            and dy2.is_contiguous() and x2.shape[1] % 8 == 0 and dy2.shape[1] % 8 == 0 and dy2.shape[1] <= 8192
            and x2.shape[0] >= 1024 and x2.shape[0] < (1 << 31) and x2.data_ptr() % 16 == 0
            and dy2.data_ptr() % 16 == 0)


# workgroups the 256x256 kernel's split-K aims at (one per CU: 128 KiB of LDS each)
WG256_TARGET = 256


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype, splits: int | None = None) -> torch.Tensor:
    """``dy2^T @ x2`` ([N_out, N_in]) on the split-K HIP kernels (bf16 operands, fp32 accumulation):
    the 256x256-tile kernel (``wgrad256.hip``) when both widths are multiples of 256, else the
    128x128 one (``gemm_glds.hip``)."""
    from .gemm import conv1x1_wgrad_v2

    K, n_out = dy2.shape
    n_in = x2.shape[1]
    C = _ext.get(required=True)
    if C.wgrad256_supported(n_out, n_in, K, dy2.stride(0),
                                                                                  x2.stride(0)):
        tiles = (n_out // 256) * (n_in // 256)
        # exactly one round of workgroups (floor, not ceil: a second, partial round costs a whole
        # round — fc1 7 splits x 36 tiles = 252 workgroups ran in 245 us, 8 x 36 = 288 in 375 us)
        s = splits or max(1, min(WG256_TARGET // tiles, K // 512))
        s = C.wgrad256_actual_splits(K, s)
        ws = torch.empty(s, n_out, n_in, device=dy2.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(dy2.device).cuda_stream
        C.gemm_wgrad256(dy2.data_ptr(), x2.data_ptr(), ws.data_ptr(), dy2.stride(0), x2.stride(0), n_out, n_in, K, s,
                        stream)
        odt = out_dtype if out_dtype in (torch.float32, torch.bfloat16) else torch.float32
        dw = graddst.empty((n_out, n_in), odt, dy2.device)
        C.gemm_splitk_reduce(ws.data_ptr(), s, dw.numel(), dw.data_ptr(), DTYPE_CODE[odt], stream)
        return dw.to(out_dtype)
    return conv1x1_wgrad_v2(dy2, x2, out_dtype=out_dtype, splits=splits or _SPLITS.get((n_out, n_in)))


# One launch for a Linear's input AND weight gradient (csrc/kernels/linbwd.hip); "0": the two
# separate calls (dgrad below + weight_grad)
LINBWD = os.environ.get("FLUXMPI_LINBWD", "1") != "0"


def linbwd_candidates(M: int, N: int, K: int, cus: int) -> tuple[list, int]:
    """Split counts the one-launch backward is timed at (weight-gradient jobs between a quarter
    and all of the CUs' worth, four geometric steps) and the untimed default (about half)."""
    C = _ext.get(required=True)
    tiles = max(1, (N // 256) * (K // 256))
    lo, hi = max(1, cus // 4 // tiles), max(1, cus // tiles)
    raw = {max(1, round(lo * (hi / lo) ** (i / 3))) for i in range(4)} if hi > lo else {lo}
    cands = sorted({C.linear_bwd_splits(M, N, K, min(64, sp)) for sp in raw})
    return cands, C.linear_bwd_splits(M, N, K, max(1, min(64, cus // 2 // tiles)))


def linbwd_ok(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor) -> bool:
    if not (LINBWD and dy2.is_cuda and dy2.dtype == x2.dtype == w.dtype == torch.bfloat16):
        return False
    if not (dy2.is_contiguous() and x2.is_contiguous() and w.is_contiguous()):
        return False
    if any(t.data_ptr() % 16 for t in (dy2, x2, w)):
        return False
    C = _ext.get(required=False)
    if C is None or not hasattr(C, "linear_bwd"):
        return False
    M, N = dy2.shape
    K = x2.shape[1]
    return tuple(w.shape) == (N, K) and bool(C.linear_bwd_supported(M, N, K, N, K, K, K))


def _lb_known():
    from .conv_choice import _LB_CHOICE
    return _LB_CHOICE


def dgrad_wgrad(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, out_dtype: torch.dtype):
    """``(dy2 @ w, dy2^T @ x2)`` — a Linear's input and weight gradients — in ONE launch of
    ``linbwd.hip`` (fp32 accumulation; the weight gradient's split-K partials reduced into
    ``out_dtype``, into the weight's DDP bucket slice when the caller binds it with
    ``graddst.into``). The split count is measured once per shape among
    :func:`linbwd_candidates` (``ops/conv_choice.linbwd_choice``: rank-consistent through
    ``parallel/autotune.calibrate``); on the ViT-B/16 shapes the best points lie at 108-144
    weight-gradient jobs, weight gradient first: qkv 334-341 us, proj 128-131, fc1 434-451
    against 363 / 148 / 444-450 for hipBLASLt's input gradient + wgrad256, and the cost is not
    smooth in the split count (qkv 5 splits 364 us), so it is timed, not modelled. Callers check
    :func:`linbwd_ok` first."""
    from .conv_choice import linbwd_choice
    C = _ext.get(required=True)
    M, N = dy2.shape
    K = x2.shape[1]
    cus = torch.cuda.get_device_properties(dy2.device).multi_processor_count
    stream = torch.cuda.current_stream(dy2.device).cuda_stream
    dx = torch.empty(M, K, device=dy2.device, dtype=dy2.dtype)
    cands, default = linbwd_candidates(M, N, K, cus)

    def trial(sp):  # into scratch: a measured launch never touches the real outputs
        C.linear_bwd(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), dx.data_ptr(), scratch.data_ptr(), M, N, K, N, K,
                     K, K, sp, 0, stream)

    scratch = None
    if (M, N, K, cus) not in _lb_known():
        scratch = torch.empty(max(cands + [default]), N, K, device=dy2.device, dtype=torch.float32)
    sp = linbwd_choice((M, N, K, cus), cands, default, trial)
    del scratch
    ws = torch.empty(sp, N, K, device=dy2.device, dtype=torch.float32)
    # weight-gradient jobs first (the longer jobs; the input-gradient tiles fill the tail):
    # measured 8-25 % faster than the other order at every split count (profiles/rd6d_bench_linbwd.jsonl)
    C.linear_bwd(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), dx.data_ptr(), ws.data_ptr(), M, N, K, N, K, K, K, sp,
                 0, stream)
    odt = out_dtype if out_dtype in (torch.float32, torch.bfloat16) else torch.float32
    dw = graddst.empty((N, K), odt, dy2.device)
    C.gemm_splitk_reduce(ws.data_ptr(), sp, dw.numel(), dw.data_ptr(), DTYPE_CODE[odt], stream)
    return dx, dw.to(out_dtype)


def bias_grad(dy2: torch.Tensor, out_dtype: torch.dtype) -> torch.Tensor:
    """Column sums of ``dy2`` [rows, N] -> [N] (fp32 accumulation, cast to ``out_dtype``)."""
    if not (dy2.is_cuda and dy2.dtype in DTYPE_CODE and dy2.is_contiguous() and dy2.shape[1] % 8 == 0
            and dy2.shape[1] <= 8192 and dy2.data_ptr() % 16 == 0):
        return dy2.float().sum(0).to(out_dtype)
    C = _ext.get(required=True)
    rows, n = dy2.shape
    stream = torch.cuda.current_stream(dy2.device).cuda_stream
    from .attention import take_colpart
    part = take_colpart(dy2)  # dQKV of the packed attention: its kernels left the partial sums
    if part is not None:
        blocks = part.shape[0]
    else:
        blocks = C.colsum_blocks(rows)
        part = torch.empty(blocks, n, device=dy2.device, dtype=torch.float32)
        C.colsum(dy2.data_ptr(), part.data_ptr(), blocks, rows, n, DTYPE_CODE[dy2.dtype], stream)
    odt = out_dtype if out_dtype in (torch.float32, torch.bfloat16) else torch.float32
    db = graddst.empty((n,), odt, dy2.device)
    C.gemm_splitk_reduce(part.data_ptr(), blocks, n, db.data_ptr(), DTYPE_CODE[odt], stream)
    return db.to(out_dtype)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.bias = bias  # the leaf itself (not saved data): the bias gradient's bucket slice
        return fwd(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        n_out, n_in = w.shape
        dy2 = dy.reshape(-1, n_out)
        x2 = x.reshape(-1, n_in)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dw = db = None
        native = _wgrad_mode() == "ours" and native_ok(x2, dy2)
        need_w = ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]

        # written straight into the DDP bucket slices when a communicating engine is attached
        same = dy2.dtype == x2.dtype == w.dtype
        dx = None
        if need_w and ctx.needs_input_grad[0] and native and linbwd_ok(dy2, x2, w):
            # both GEMMs in one launch (linbwd.hip): the weight gradient's jobs fill the input
            # gradient's partial last round
            with graddst.into(w):
                dx, dw = dgrad_wgrad(dy2, x2, w, w.dtype)
            dx = dx.reshape(x.shape)
            need_w = False
        if need_w:
            def wgrad():
                with graddst.into(w):
                    if native:
                        return weight_grad(dy2, x2, w.dtype)
                    if same:  # short K (e.g. a classifier head): hipBLASLt, output in the slice
                        return torch.mm(dy2.t(), x2, out=graddst.empty(tuple(w.shape), w.dtype, dy2.device))
                    return (dy2.t() @ x2).to(w.dtype)
            dw = wgrad()
        if need_b:
            with graddst.into(ctx.bias):
                if native:
                    db = bias_grad(dy2, ctx.bias_dtype)
                elif dy2.dtype == ctx.bias_dtype:
                    db = torch.sum(dy2, 0, out=graddst.empty((n_out,), ctx.bias_dtype, dy2.device))
                else:
                    db = dy2.sum(0).to(ctx.bias_dtype)
        if dx is None and ctx.needs_input_grad[0]:
            dx = dgrad(dy2, w).reshape(x.shape)
        return dx, dw, db


def fwd(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """``F.linear`` — on gemm_nt.hip (bias in the epilogue) when the shape tiles exactly."""
    from . import gemm_nt
    n_out, n_in = weight.shape
    rows = x.numel() // n_in if n_in else 0
    if x.is_contiguous() and gemm_nt.supported(rows, n_out, n_in, x, weight, fused="plain_fwd"):
        return gemm_nt.linear_fwd(x.view(rows, n_in), weight, bias).view(*x.shape[:-1], n_out)
    return F.linear(x, weight, bias)


def dgrad(dy2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``dy2 [rows, N_out] @ weight [N_out, N_in]`` — on gemm_nt.hip (over W^T) when the shape tiles."""
    from . import gemm_nt
    n_out, n_in = weight.shape
    if dy2.is_contiguous() and gemm_nt.supported(dy2.shape[0], n_in, n_out, dy2, weight):
        return gemm_nt.linear_dgrad(dy2, weight)
    return dy2 @ weight


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear`` with the HIP weight/bias-gradient backward for bf16 token-major inputs."""
    if x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled() and weight.requires_grad:
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class Linear(torch.nn.Linear):
    """Drop-in ``nn.Linear`` whose backward uses :func:`linear`'s kernels."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)


__all__ = ["linear", "Linear", "weight_grad", "bias_grad", "native_ok", "fwd", "dgrad", "dgrad_wgrad", "linbwd_ok"]
