"""Token-major Linear GEMMs on the ping-pong 256x256 NT kernel (``csrc/kernels/gemm_nt.hip``).

* :func:`linear_fwd` — ``y = x W^T + b`` (``gelu=True``: ``gelu(y)`` and ``gelu'(y)`` instead,
  from the same registers: fc1 of a transformer MLP writes its activation and the derivative
  its backward needs in one pass, no elementwise GELU kernel);
* :func:`linear_dgrad` — ``dx = dy W`` on ``W^T`` (one ``transpose_bf16`` of the 0.6-4.7 MB
  weight per call, so both operands of the GEMM stay k-contiguous); ``gelu_d=gelu'(h)``:
  ``dh = dx * gelu'(h)`` and the column sums of ``dh`` — the previous Linear's bias gradient,
  written into its DDP bucket slice when one is attached (``ops/graddst.py``) — in the epilogue.

The ViT-B/16 Linears at batch 256 (M = 50432 = 197 x 256 tokens, N and K in {768, 2304, 3072})
tile exactly; :func:`supported` says whether a call qualifies, callers keep the PyTorch path
otherwise. Numerics: bf16 operands, fp32 accumulation, one bf16 rounding of each output (the
GELU of the ROUNDED pre-activation, like ``F.gelu(F.linear(...))``); the saved derivative is
bf16 too, so ``dh`` carries one extra bf16 rounding of ``gelu'(h)`` compared with autograd's
fp32 derivative (relative error <= 2^-9 per element, below the output's own rounding).

``FLUXMPI_GEMM_NT``: ``fused`` (default) the calls that carry an epilogue fusion — fc1's bias +
GELU forward (EPI 1: gelu(h) and gelu'(h) from one tanh evaluation; the derivative replaces the
pre-activation as what the backward saves) and fc2's input gradient times that derivative +
fc1's bias-gradient partials (EPI 2: no GELU math left in the backward); ``all`` also every
plain forward / input gradient (at parity with hipBLASLt on qkv / proj, 1-5 % behind on the
K = 3072 / N = 3072 ones); ``fwd`` the fused calls and every plain forward (the input gradients of
the plain Linears go to ``linbwd.hip`` either way, ``ops/linear.py``); ``0`` never. Measured: profiles/rd4i_bench_gemm_nt.jsonl (the hipBLASLt
columns are the roofline baseline per shape).

Convolutions (ops/gemm.py routes here, ``FLUXMPI_GEMM_NT_CONV``, default on): the stride-1 3x3
forward / input gradient and the 1x1 forward / input gradient when the output has >= 160 tiles
(a persistent workgroup per CU needs them) and K >= 1024 — where the 256x256 tiles beat the
128-tile kernel: 3x3 at 14x14x256 70 vs 101 us; short K or few tiles lose
(profiles/rd4f_bench_conv_nt.jsonl).
"""
from __future__ import annotations

import os

import torch

from . import _ext
from . import graddst
from .multi_tensor import DTYPE_CODE

MODE = os.environ.get("FLUXMPI_GEMM_NT", "fused").lower()
ENABLED = MODE != "0"
# In the default ("fused") mode a plain Linear forward also runs here when its K is at most this
# (ViT-B/16's qkv and proj at 1024). Default 0 (none), by measurement: qkv + proj on gemm_nt take
# the same kernel time as hipBLASLt (2.98 vs ~2.95 ms/step, profiles/rd6z_vit_b16_steady.md) and
# cut hipBLASLt to fc2 (2.75 ms), but ViT-B/16 measured -0.4 % in three interleaved pairs
# (profiles/rd6z_vit_plain_fwd_ab.jsonl); plain forward GEMMs stay on the vendor library.
PLAIN_FWD_MAX_K = int(os.environ.get("FLUXMPI_GEMM_NT_PLAIN_FWD_MAX_K", "0"))


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _aligned(*tensors: torch.Tensor) -> bool:
    """The kernels' buffer resources and 16-B vector accesses need 16-B aligned operands (an
    oddly offset view, e.g. a narrowed buffer, routes to the fallback instead of raising)."""
    return all(t.data_ptr() % 16 == 0 for t in tensors)


def supported(rows: int, n_out: int, k: int, *tensors: torch.Tensor, fused: bool | str = False) -> bool:
    """Whether gemm_nt takes ``[rows, k] x [n_out, k]^T`` (both operands k-contiguous after the
    weight transpose of an input gradient) under the current mode. ``fused``: the call carries an
    epilogue fusion — ``"fwd"`` (fc1 bias + GELU) or ``"dgrad"`` (GELU backward), taken in modes
    fused / all (the pair works together: the backward multiplies by the derivative the forward
    stored), ``True`` (either: shape checks of the kernel itself), ``"plain_fwd"`` (a plain Linear
forward: taken in modes fwd / all, and in the default mode up to :data:`PLAIN_FWD_MAX_K`)."""
    if not ENABLED or not tensors or not tensors[0].is_cuda:
        return False
    if MODE not in ("all", "1"):
        ok = (fused is True or (fused in ("fwd", "dgrad") and MODE in ("fused", "dgrad", "fwd"))
              or (fused == "plain_fwd" and (MODE == "fwd" or (MODE == "fused" and k <= PLAIN_FWD_MAX_K))))
        if not ok:
            return False
    if any(t.dtype != torch.bfloat16 for t in tensors) or not _aligned(*tensors):
        return False
    C = _ext.get(required=False)
    return C is not None and hasattr(C, "gemm_nt") and bool(C.gemm_nt_supported(rows, n_out, k, k, k, n_out))


def _set_split(min_ktiles: int) -> None:
    """TEST / DIAGNOSTIC knob, not public API (its EPI 2 fix-up path needed the epilogue store guard,
    root cause not pinned: profiles/rd6_store_hazard_scan.md). The split-K tail of the persistent kernel (``FLUXMPI_GEMM_NT_SPLIT``, default 0 = off: measured slower end to end, profiles/rd5d_*): the last,
    partial round of each XCD's tiles is cut into even k-tile ranges of at least ``min_ktiles``
    spread over all its workgroups (pieces summed by the last arriving workgroup, in piece order:
    deterministic); ``0`` runs the last round tile-granular."""
    _ext.get(required=True).gemm_nt_set_split(int(min_ktiles))


def get_split() -> int:
    """The split-K tail setting in force (see :func:`_set_split`)."""
    return int(_ext.get(required=True).gemm_nt_get_split())


def weight_t(weight: torch.Tensor) -> torch.Tensor:
    """``weight.t().contiguous()`` by the 16-B-vector transpose kernel."""
    C = _ext.get(required=True)
    w = weight.contiguous()
    r, c = w.shape
    wt = torch.empty(c, r, device=w.device, dtype=w.dtype)
    C.transpose_bf16(w.data_ptr(), wt.data_ptr(), r, c, c, r, _stream(w))
    return wt


def linear_fwd(x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, gelu: bool = False):
    """``x2 [M, K] @ weight[N, K]^T + bias`` -> ``y [M, N]`` (bf16); ``gelu``: ``(gelu'(y), gelu(y))``
    — the derivative is what the backward multiplies by (:func:`linear_dgrad`'s ``gelu_d``), so
    the pre-activation ``y`` itself is never written."""
    C = _ext.get(required=True)
    m, k = x2.shape
    n = weight.shape[0]
    x2 = x2.contiguous()
    w = weight.contiguous()
    y = torch.empty(m, n, device=x2.device, dtype=x2.dtype)
    g = torch.empty_like(y) if gelu else None
    if gelu:
        from .gelu import _sync
        _sync(C)  # EPI 1 computes the selected GELU form
    b = bias.contiguous() if bias is not None else None
    s = _stream(x2)
    C.gemm_nt(x2.data_ptr(), w.data_ptr(), y.data_ptr(), g.data_ptr() if gelu else 0,
              b.data_ptr() if b is not None else 0, int(b is not None and b.dtype == torch.float32), 0, 0,
              k, k, n, m, n, k, 1 if gelu else 0, s)
    return (y, g) if gelu else y


def linear_dgrad(dy2: torch.Tensor, weight: torch.Tensor, gelu_d: torch.Tensor | None = None,
                 bias_dtype=torch.float32, bias_param: torch.Tensor | None = None):
    """``dy2 [M, N] @ weight [N, K]`` -> ``dx [M, K]``. With ``gelu_d`` (``gelu'(h)`` of the GELU
    that produced this Linear's input, ``[M, K]``, as :func:`linear_fwd` stored it): returns
    ``(dh, db)`` with ``dh = bf16(dx) * gelu'(h)`` and ``db = dh.sum(0)`` in ``bias_dtype``
    (delivered into ``bias_param``'s bucket slice)."""
    C = _ext.get(required=True)
    m, n = dy2.shape
    k = weight.shape[1]
    dy2 = dy2.contiguous()
    wt = weight_t(weight)  # [K][N]: the B operand, k(= N)-contiguous
    dx = torch.empty(m, k, device=dy2.device, dtype=dy2.dtype)
    s = _stream(dy2)
    if gelu_d is None:
        C.gemm_nt(dy2.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0, n, n, k, m, k, n, 0, s)
        return dx
    h = gelu_d.reshape(m, k).contiguous()
    rows = C.gemm_nt_colpart_rows(m)
    part = torch.empty(rows, k, device=dy2.device, dtype=torch.float32)
    C.gemm_nt(dy2.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, 0, 0, h.data_ptr(), part.data_ptr(),
              n, n, k, m, k, n, 2, s)
    odt = bias_dtype if bias_dtype in (torch.float32, torch.bfloat16) else torch.float32
    with graddst.into(bias_param):
        db = graddst.empty((k,), odt, dy2.device)
    C.gemm_splitk_reduce(part.data_ptr(), rows, k, db.data_ptr(), DTYPE_CODE[odt], s)
    return dx, db.to(bias_dtype)


# convolutions on the same kernel (ops/gemm.py routes to these): "1" (default) wherever a shape
# qualifies, "0" never
CONV = os.environ.get("FLUXMPI_GEMM_NT_CONV", "1") != "0"


MIN_TILES = 160
MIN_K = 1024


def _worth(rows: int, n_out: int, k: int) -> bool:
    return (rows // 256) * (n_out // 256) >= MIN_TILES and k >= MIN_K


def conv_ok(pixels: int, c: int, cout: int, *tensors: torch.Tensor) -> bool:
    """Whether a 3x3 / stride 1 / pad 1 convolution over ``pixels`` output pixels (C -> Cout)
    runs on :func:`conv3x3`."""
    if not CONV or not tensors or not tensors[0].is_cuda or any(t.dtype != torch.bfloat16 for t in tensors):
        return False
    if not _aligned(*tensors) or not _worth(pixels, cout, 9 * c):
        return False
    C = _ext.get(required=False)
    return C is not None and hasattr(C, "gemm_nt_conv") and bool(C.gemm_nt_conv_supported(pixels, c, cout))


def gemm_ok(rows: int, n_out: int, k: int, *tensors: torch.Tensor) -> bool:
    """Whether a 1x1 convolution / plain NT GEMM of this shape runs on :func:`gemm_plain`."""
    if not CONV or not tensors or not tensors[0].is_cuda or any(t.dtype != torch.bfloat16 for t in tensors):
        return False
    if not _aligned(*tensors) or not _worth(rows, n_out, k):
        return False
    C = _ext.get(required=False)
    return C is not None and hasattr(C, "gemm_nt_stats") and bool(C.gemm_nt_supported(rows, n_out, k, k, k, n_out))


def conv3x3(x: torch.Tensor, w_taps: torch.Tensor, y: torch.Tensor, stats: torch.Tensor | None = None,
            residual: torch.Tensor | None = None) -> torch.Tensor:
    """``y [N*H*W, Cout] = conv3x3(x)``: ``x`` NHWC [N, H, W, C] memory (a channels_last tensor),
    ``w_taps`` [Cout, 9*C] (tap-major, channel-fastest: a channels_last filter, or the flipped
    transpose of the input-gradient), ``stats``: the BatchNorm shards [64, 2, Cout] receive the
    output's per-channel sum / sum of squares (EPI 3); ``residual`` (laid out as ``y``, 16-B
    aligned): ``y = bf16(bf16(conv) + residual)`` (EPI 4; not with ``stats``)."""
    C = _ext.get(required=True)
    n, c, h, wd = x.shape
    cout = w_taps.shape[0]
    s = _stream(x)
    assert stats is None or residual is None
    epi = 3 if stats is not None else (4 if residual is not None else 0)
    C.gemm_nt_conv(x.data_ptr(), w_taps.data_ptr(), y.data_ptr(), stats.data_ptr() if stats is not None else 0,
                   n, h, wd, c, cout, epi, s, residual.data_ptr() if residual is not None else 0)
    return y


def gemm_plain(a2: torch.Tensor, b2: torch.Tensor, c2: torch.Tensor, stats: torch.Tensor | None = None) -> torch.Tensor:
    """``c2 [M, N] = a2 [M, K] @ b2 [N, K]^T`` (both k-contiguous rows); ``stats`` as in :func:`conv3x3`."""
    C = _ext.get(required=True)
    m, k = a2.shape
    n = b2.shape[0]
    s = _stream(a2)
    if stats is not None:
        C.gemm_nt_stats(a2.data_ptr(), b2.data_ptr(), c2.data_ptr(), stats.data_ptr(), a2.stride(0), b2.stride(0),
                        c2.stride(0), m, n, k, s)
    else:
        C.gemm_nt(a2.data_ptr(), b2.data_ptr(), c2.data_ptr(), 0, 0, 0, 0, 0, a2.stride(0), b2.stride(0),
                  c2.stride(0), m, n, k, 0, s)
    return c2


__all__ = ["supported", "weight_t", "linear_fwd", "linear_dgrad", "conv_ok", "gemm_ok", "conv3x3", "gemm_plain",
           "ENABLED", "MODE", "CONV"]
