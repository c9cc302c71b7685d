"""Anderson-acceleration solver ops for the DEQ fixed-point solve (``csrc/kernels/anderson.hip``).

The solver history ``X, F`` is ``[bsz, m, d]`` fp32. Every iteration needs the Gram matrix
``G G^T`` of ``G = F[:, :n] - X[:, :n]`` and the mix ``X[:, s] = beta * alpha F + (1 - beta)
* alpha X``. On the GPU both are single streaming HIP passes (G formed in registers, the
new iterate's model-dtype copy written by the mix); CPU tensors use the PyTorch
composition, which is also the test oracle.
"""
from __future__ import annotations

import torch

from . import _ext
from .multi_tensor import DTYPE_CODE

_MAX_ROWS = 8
_SYM_IDX: dict = {}


def _sym_index(n: int, device) -> torch.Tensor:
    """[n*n] positions in the packed upper-triangle order of the Gram kernel: H = tot[:, idx]."""
    key = (n, str(device))
    t = _SYM_IDX.get(key)
    if t is None:
        iu = torch.triu_indices(n, n)
        pos = torch.empty(n, n, dtype=torch.long)
        pos[iu[0], iu[1]] = torch.arange(iu.shape[1])
        pos[iu[1], iu[0]] = torch.arange(iu.shape[1])
        t = _SYM_IDX[key] = pos.reshape(-1).to(device)
    return t


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _native(X: torch.Tensor, F: torch.Tensor, n: int) -> bool:
    if not (X.is_cuda and F.is_cuda):
        return False
    ok = (X.dtype in (torch.float32, torch.bfloat16) and F.dtype in (torch.float32, torch.bfloat16)
          and X.dim() == F.dim() == 3
          and X.shape == F.shape
          and X.stride() == F.stride() and X.stride(2) == 1 and X.shape[2] % 4 == 0 and X.stride(1) % 4 == 0
          and X.stride(0) % 4 == 0 and 1 <= n <= min(_MAX_ROWS, X.shape[1]) and X.shape[0] <= 65535
          and X.data_ptr() % 16 == 0 and F.data_ptr() % 16 == 0)
    if not ok:
        raise ValueError("anderson ops: need fp32 / bf16 X and F histories [bsz<=65535, m, d%4==0] with "
                         "matching strides, n<=8")
    return True


def gram(X: torch.Tensor, F: torch.Tensor, n: int, last: int, G: torch.Tensor | None = None, fresh=None):
    """``(G G^T [bsz, n, n], |F[:, last]|^2 [bsz])`` with ``G = F[:, :n] - X[:, :n]`` (fp32).

    ``G`` (optional, same shape/strides as X): stored differences. Rows listed in ``fresh``
    are recomputed from ``F - X`` and written to ``G``; the others are read from ``G``
    (an iteration that changed one row reads 2 + (n - 1) rows instead of 2n)."""
    if not _native(X, F, n):
        if G is not None:
            for i in fresh:
                G[:, i] = F[:, i].float() - X[:, i].float()
            Gn = G[:, :n].float()
        else:
            Gn = F[:, :n].float() - X[:, :n].float()
        return torch.bmm(Gn, Gn.transpose(1, 2)), F[:, last].float().pow(2).sum(1)
    C = _ext.get(required=True)
    bsz, _, d = X.shape
    chunks = C.anderson_gram_chunks(bsz, d)
    part = torch.empty(bsz, chunks, 37, device=X.device, dtype=torch.float32)
    mask = 0
    if G is not None:
        if G.shape != X.shape or G.stride() != X.stride() or G.dtype != X.dtype or G.data_ptr() % 16:
            raise ValueError("anderson gram: G must match X's shape, strides and dtype")
        for i in fresh:
            mask |= 1 << int(i)
    C.anderson_gram(X.data_ptr(), F.data_ptr(), DTYPE_CODE[F.dtype], G.data_ptr() if G is not None else 0, mask,
                    part.data_ptr(), bsz, d, X.stride(1), X.stride(0), n, last, chunks, _stream(X), DTYPE_CODE[X.dtype])
    tot = part.sum(1)
    # one gather (cached symmetric index) instead of building the index and two scatters
    H = tot.index_select(1, _sym_index(n, X.device)).view(bsz, n, n)
    return H, tot[:, 36]


def gram_solve(X: torch.Tensor, F: torch.Tensor, n: int, last: int, G: torch.Tensor, fresh, lam: float,
               want_res: bool, res_out: torch.Tensor | None = None):
    """``(alpha [bsz, n], res)`` of one Anderson step: the Gram pass (:func:`gram`, stored ``G``)
    then ONE launch (``anderson_solve``) for the chunk sums, the relative residual of row ``last``
    (a 0-d device tensor, or None without ``want_res``) and the batched pivoted solve of
    ``[[0, 1^T], [1, G G^T + lam I]] a = e_0``, ``alpha = a[1:]``. CPU tensors (and batches over
    1024) use the PyTorch composition: :func:`gram`, ``torch.linalg.solve_ex``.
    ``res_out`` (0-d fp32 device tensor, with ``want_res``): the residual is written there (no copy
    of a fresh scalar into the caller's buffer)."""
    bsz = X.shape[0]
    if not (_native(X, F, n) and bsz <= 1024):
        H, fn2 = gram(X, F, n, last, G, fresh)
        res = (H[:, last, last].sum().sqrt() / (1e-5 + fn2.sum().sqrt())) if want_res else None
        if res is not None and res_out is not None:
            res_out.copy_(res)
            res = res_out
        A = torch.zeros(bsz, n + 1, n + 1, dtype=torch.float32, device=X.device)
        A[:, 0, 1:] = A[:, 1:, 0] = 1
        A[:, 1:, 1:] = H + lam * torch.eye(n, dtype=torch.float32, device=X.device)
        y = torch.zeros(bsz, n + 1, 1, dtype=torch.float32, device=X.device)
        y[:, 0] = 1
        return torch.linalg.solve_ex(A, y, check_errors=False)[0][:, 1:, 0], res
    C = _ext.get(required=True)
    d = X.shape[2]
    chunks = C.anderson_gram_chunks(bsz, d)
    part = torch.empty(bsz, chunks, 37, device=X.device, dtype=torch.float32)
    if G.shape != X.shape or G.stride() != X.stride() or G.dtype != X.dtype or G.data_ptr() % 16:
        raise ValueError("anderson gram: G must match X's shape, strides and dtype")
    mask = 0
    for i in fresh:
        mask |= 1 << int(i)
    stream = _stream(X)
    C.anderson_gram(X.data_ptr(), F.data_ptr(), DTYPE_CODE[F.dtype], G.data_ptr(), mask, part.data_ptr(), bsz, d,
                    X.stride(1), X.stride(0), n, last, chunks, stream, DTYPE_CODE[X.dtype])
    alpha = torch.empty(bsz, n, device=X.device, dtype=torch.float32)
    res = (res_out if res_out is not None else torch.empty((), device=X.device, dtype=torch.float32)) \
        if want_res else None
    C.anderson_solve(part.data_ptr(), chunks, bsz, n, last, float(lam), alpha.data_ptr(),
                     res.data_ptr() if res is not None else 0, stream)
    return alpha, res


def mix(X: torch.Tensor, F: torch.Tensor, alpha: torch.Tensor, slot: int, beta: float = 1.0,
        z_dtype: torch.dtype | None = None):
    """``X[:, slot] = beta * alpha F[:, :n] + (1 - beta) * alpha X[:, :n]`` in place (n = alpha.shape[1]).

    Returns the new iterate as a ``[bsz, d]`` tensor of ``z_dtype`` (a fresh copy when it is not fp32;
    the ``X[:, slot]`` view otherwise)."""
    n = alpha.shape[1]
    if not _native(X, F, n):
        new = beta * torch.bmm(alpha[:, None], F[:, :n].float())[:, 0]
        if beta != 1.0:
            new = new + (1 - beta) * torch.bmm(alpha[:, None], X[:, :n].float())[:, 0]
        X[:, slot] = new
        return X[:, slot] if z_dtype in (None, X.dtype) else new.to(z_dtype)
    C = _ext.get(required=True)
    bsz, _, d = X.shape
    a = alpha.float().contiguous()
    z = None
    if z_dtype not in (None, torch.float32):
        z = torch.empty(bsz, d, device=X.device, dtype=z_dtype)
    C.anderson_mix(X.data_ptr(), F.data_ptr(), DTYPE_CODE[F.dtype], a.data_ptr(), z.data_ptr() if z is not None else 0,
                   DTYPE_CODE[z_dtype] if z is not None else 7, bsz, d, X.stride(1), X.stride(0), n, slot, float(beta),
                   _stream(X), DTYPE_CODE[X.dtype])
    return z if z is not None else X[:, slot]


def adjoint_step(vjp: torch.Tensor, grad: torch.Tensor, u: torch.Tensor, out: torch.Tensor | None = None,
                 thresh2: torch.Tensor | None = None, flag: torch.Tensor | None = None):
    """``(u_new, ss)``: ``u_new = vjp + grad`` and ``ss = |u_new - u|^2`` (0-d fp32 device tensor)
    in one pass on the GPU (``adjoint_step`` + one partial-sum reduce); the DEQ adjoint solve's
    update and convergence test. ``out`` (optional, like ``vjp``, not ``u``): written instead of a
    new tensor. ``thresh2`` / ``flag`` (fp32 device scalar / one fp32 element): also
    ``flag = ss <= thresh2``, in the reduce's launch on the GPU (no compare / cast / copy kernels per
    iteration). Other layouts / CPU: the PyTorch composition."""
    same = (vjp.shape == grad.shape == u.shape and vjp.dtype == grad.dtype == u.dtype
            and vjp.stride() == grad.stride() == u.stride())
    dense = same and vjp.numel() % 8 == 0 and (vjp.is_contiguous() or (vjp.dim() == 4 and vjp.is_contiguous(
        memory_format=torch.channels_last)))
    if not (vjp.is_cuda and dense and vjp.dtype in DTYPE_CODE and vjp.numel() > 0
            and (vjp.data_ptr() | grad.data_ptr() | u.data_ptr()) % 16 == 0):
        u_new = torch.add(vjp, grad, out=out) if out is not None else vjp + grad
        ss = (u_new - u).float().pow(2).sum()
        if flag is not None:
            flag.copy_((ss <= thresh2).float().reshape(flag.shape))
        return u_new, ss
    C = _ext.get(required=True)
    n = vjp.numel()
    blocks = C.adjoint_step_blocks(n)
    # same strides (dense), so the flat element order matches
    u_new = out if (out is not None and out.stride() == vjp.stride() and out.dtype == vjp.dtype) else \
        torch.empty_like(vjp)
    part = torch.empty(blocks, device=vjp.device, dtype=torch.float32)
    ss = torch.empty((), device=vjp.device, dtype=torch.float32)
    stream = _stream(vjp)
    C.adjoint_step(vjp.data_ptr(), grad.data_ptr(), u.data_ptr(), u_new.data_ptr(), part.data_ptr(), blocks, n,
                   DTYPE_CODE[vjp.dtype], stream)
    if flag is not None:
        if not (thresh2 is not None and thresh2.dtype == flag.dtype == torch.float32 and flag.is_contiguous()
                and thresh2.is_cuda and flag.is_cuda and flag.numel() == 1):
            raise ValueError("adjoint_step: flag needs a one-element fp32 flag and an fp32 device thresh2")
        C.deq_adjoint_check(part.data_ptr(), blocks, thresh2.data_ptr(), ss.data_ptr(), flag.data_ptr(), stream)
    else:
        C.gemm_splitk_reduce(part.data_ptr(), blocks, 1, ss.data_ptr(), DTYPE_CODE[torch.float32], stream)
    return u_new, ss
