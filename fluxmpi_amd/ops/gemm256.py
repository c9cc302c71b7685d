"""Token-major Linear GEMMs on 256 x 256 tiles with fused epilogues (``csrc/kernels/gemm256.hip``).

* :func:`linear_fwd` — ``y = x W^T + b`` (``gelu=True``: also ``g = gelu(y)``, the ops.gelu form,
  from the same registers: fc1 of a transformer MLP writes its pre-activation and its
  activation in one pass, no elementwise GELU kernel);
* :func:`linear_dgrad` — ``dx = dy W`` (``gelu_h=h``: ``dh = dx * gelu'(h)`` and the column
  sums of ``dh`` — the previous Linear's bias gradient — in the epilogue, no gelu_bwd_bias
  pass).

Shapes must tile exactly (rows and output columns multiples of 256: ViT-B/16 has 50432 =
197 x 256 tokens at batch 256); :func:`supported` says whether a call qualifies, callers keep
the PyTorch path otherwise. Numerics: bf16 operands, fp32 accumulation, one bf16 rounding of
each output (the GELU of the ROUNDED pre-activation, like ``F.gelu(F.linear(...))``).
"""
from __future__ import annotations

import os

import torch

from . import _ext
from .multi_tensor import DTYPE_CODE

# Which calls take gemm256 (FLUXMPI_GEMM256):
#   "fused" (default): only the epilogue fusions measured faster than hipBLASLt + the separate pass
#            they replace — fc2's input gradient with the GELU backward and fc1's bias gradient
#            (409 us vs 242 + 197 us per ViT-B/16 block, profiles/rd3d_bench_gemm256.jsonl);
#   "all":   also the plain forward / input gradient and fc1's bias + GELU forward (our main loop
#            runs 0.59-0.87 PF/s against hipBLASLt's 0.92-1.12 on these shapes: not yet a win);
#   "0":     never.
MODE = os.environ.get("FLUXMPI_GEMM256", "fused").lower()
ENABLED = MODE != "0"


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def supported(rows: int, n_out: int, k: int, *tensors: torch.Tensor, b_t: bool = False,
              fused: bool = False) -> bool:
    """Whether gemm256 takes this call: the shape tiles exactly and the mode selects it
    (``fused``: the call carries an epilogue fusion, see ``MODE``)."""
    if not ENABLED or not tensors or not tensors[0].is_cuda:
        return False
    if MODE != "all" and not (fused and MODE == "fused"):
        return False
    if any(t.dtype != torch.bfloat16 for t in tensors):
        return False
    C = _ext.get(required=False)
    return C is not None and hasattr(C, "gemm256") and bool(C.gemm256_supported(rows, n_out, k, k, n_out if b_t else k,
                                                                                    n_out, b_t))


def linear_fwd(x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, gelu: bool = False):
    """``x2 [M, K] @ weight[N, K]^T + bias`` -> ``y [M, N]`` (bf16); ``gelu``: ``(y, gelu(y))``."""
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
    C.gemm256(x2.data_ptr(), w.data_ptr(), y.data_ptr(), g.data_ptr() if gelu else 0,
              b.data_ptr() if b is not None else 0, int(b is not None and b.dtype == torch.float32), 0, 0,
              k, k, n, m, n, k, False, 1 if gelu else 0, _stream(x2))
    return (y, g) if gelu else y


def linear_dgrad(dy2: torch.Tensor, weight: torch.Tensor, gelu_h: torch.Tensor | None = None,
                 bias_dtype=torch.float32):
    """``dy2 [M, N] @ weight [N, K]`` -> ``dx [M, K]``. With ``gelu_h`` (the GELU input that
    produced this Linear's input, ``[M, K]``): returns ``(dh, db)`` with ``dh = dx * gelu'(h)``
    and ``db = dh.sum(0)`` in ``bias_dtype``."""
    C = _ext.get(required=True)
    m, n = dy2.shape
    k = weight.shape[1]
    dy2 = dy2.contiguous()
    w = weight.contiguous()
    dx = torch.empty(m, k, device=dy2.device, dtype=dy2.dtype)
    s = _stream(dy2)
    if gelu_h is None:
        C.gemm256(dy2.data_ptr(), w.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0, n, k, k, m, k, n, True, 0, s)
        return dx
    from .gelu import _sync
    _sync(C)  # EPI 2 differentiates the selected GELU form
    h = gelu_h.reshape(m, k).contiguous()
    rows = C.gemm256_colpart_rows(m)
    part = torch.empty(rows, k, device=dy2.device, dtype=torch.float32)
    C.gemm256(dy2.data_ptr(), w.data_ptr(), dx.data_ptr(), 0, 0, 0, h.data_ptr(), part.data_ptr(), n, k, k, m, k, n,
              True, 2, s)
    odt = bias_dtype if bias_dtype in (torch.float32, torch.bfloat16) else torch.float32
    db = torch.empty(k, device=dy2.device, dtype=odt)
    C.gemm_splitk_reduce(part.data_ptr(), rows, k, db.data_ptr(), DTYPE_CODE[odt], s)
    return dx, db.to(bias_dtype)


__all__ = ["supported", "linear_fwd", "linear_dgrad", "ENABLED", "MODE"]
