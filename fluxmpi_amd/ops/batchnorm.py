"""Fused NHWC BatchNorm(+ReLU)(+residual add) — autograd wrapper of ``csrc/kernels/batchnorm.hip``.

``FusedBatchNorm2d(C)(x, relu=True, residual=r)`` computes
``relu(batch_norm(x) + r)`` in two memory passes forward and two backward on
channels_last activations (GPU), vs ~7 / ~10 passes for the eager sequence.
Parameters and running statistics are fp32; activations may be bf16/fp16/fp32.
On CPU (and for layouts the kernels do not cover) the module runs the
PyTorch reference composition, which is also the test oracle.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import graddst
from .multi_tensor import DTYPE_CODE


def _rows_c(x: torch.Tensor):
    if x.dim() == 4:
        n, c, h, w = x.shape
        return n * h * w, c
    if x.dim() == 2:
        return x.shape[0], x.shape[1]
    raise ValueError("fused batchnorm expects 2D [N,C] or 4D [N,C,H,W] input")


def _nhwc(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 4:
        return x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(
            memory_format=torch.channels_last)
    return x.contiguous()


_WS: dict = {}
_SHARDS = 64  # == kShards in csrc/kernels/{batchnorm,gemm}.hip
_MAXC = 2048
# [_SHARDS][2][_MAXC] shards (+ 64 floats of slack)
_WS_FLOATS = _SHARDS * 2 * _MAXC + 64


def _workspace(x: torch.Tensor) -> torch.Tensor:
    """Persistent zeroed [64][2][2048] fp32 accumulator per (device, stream).

    The kernels leave it zeroed after every call (the finalize — a kernel of its own, or the
    last workgroup of the reduction kernel — re-zeroes the shards it consumes), so there is no
    memset per BatchNorm launch.
    """
    stream = torch.cuda.current_stream(x.device)
    key = (x.device.index, stream.cuda_stream)
    ws = _WS.get(key)
    if ws is None:
        ws = torch.zeros(_WS_FLOATS, device=x.device, dtype=torch.float32)
        _WS[key] = ws
    return ws


_LWS: dict = {}


def _link_workspace(x: torch.Tensor) -> torch.Tensor:
    """A second persistent zeroed accumulator, for BatchNorm-backward reductions that a GEMM
    epilogue deposits for a LATER BatchNorm backward (:class:`BNStatsLink`). Autograd may run
    another BatchNorm backward in between (e.g. a ResNet downsample branch between conv2's
    dgrad and bn1's backward), which reduces into :func:`_workspace`; keeping the linked sums
    apart makes the two independent."""
    stream = torch.cuda.current_stream(x.device)
    key = (x.device.index, stream.cuda_stream)
    ws = _LWS.get(key)
    if ws is None:
        ws = torch.zeros(_WS_FLOATS, device=x.device, dtype=torch.float32)
        _LWS[key] = ws
    return ws


_DWS: dict = {}


def _dual_workspace(x: torch.Tensor) -> torch.Tensor:
    """Third persistent zeroed accumulator: the downsample branch's sums of the dual
    (bn3 + downsample BN) backward, reduced in the same pass as bn3's into :func:`_workspace`."""
    stream = torch.cuda.current_stream(x.device)
    key = (x.device.index, stream.cuda_stream)
    ws = _DWS.get(key)
    if ws is None:
        ws = torch.zeros(_WS_FLOATS, device=x.device, dtype=torch.float32)
        _DWS[key] = ws
    return ws


def kernel_supported(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    if x.dim() not in (2, 4):
        return False
    c = x.shape[1]
    return c % 8 == 0 and 8 <= c <= 2048 and x.numel() > 0


def _grad_out(p, ch, like):
    t = graddst.take(p, (ch,), torch.float32)
    return t if t is not None else torch.empty(ch, device=like.device, dtype=torch.float32)


class GradLink:
    """Hands the residual-branch gradient of a block from the BatchNorm that adds the
    residual straight to the 1x1 convolution that also consumes the block input.

    Without it autograd sums the two gradients of the block input with a separate add
    kernel (a read-read-write pass over the largest activation of the block); with it
    the BatchNorm backward deposits ``dres`` here and the convolution's dgrad GEMM adds
    it in its epilogue. Autograd's data dependencies guarantee the order (the conv's
    backward needs gradients that pass through the BatchNorm's backward).
    """

    __slots__ = ("grad", "masked")

    def __init__(self, masked: bool = False):
        self.grad = None
        # masked: the consumer can take (dy, relu_mask) and apply the mask itself (the LDS-DMA
        # dgrad epilogue does), so the BatchNorm backward never writes dres = dy * mask
        self.masked = masked

    def take(self):
        """The residual gradient: a tensor, or ``(dy, mask)`` (1 bit per element) when masked."""
        g, self.grad = self.grad, None
        if g is None:
            raise RuntimeError("GradLink: the residual gradient was not produced before its consumer ran")
        return g


class SideGradLink:
    """Like :class:`GradLink`, for a producer that autograd does NOT order before the
    consumer by data dependency: the downsample convolution of a ResNet block, whose input
    gradient is the second summand of the block input's gradient (the first is conv1's
    dgrad). Autograd runs ready nodes newest-first, so the downsample branch (created after
    the main path) normally runs first and :meth:`offer` hands its gradient over; if the
    consumer ran first, it has closed the link and the producer returns its gradient to
    autograd as usual — correct either way, never dropped or double counted."""

    __slots__ = ("grad", "closed", "delivered")

    def __init__(self):
        self.grad = None
        self.closed = False
        self.delivered = False  # the consumer added the producer's gradient (diagnostics/tests)

    def offer(self, g: torch.Tensor) -> bool:
        if self.closed:
            return False
        self.grad = g
        return True

    def take(self):
        g, self.grad, self.closed = self.grad, None, True
        self.delivered = g is not None
        return g


class BNStatsLink:
    """Lets the kernel that produces a BatchNorm's output gradient (a dgrad GEMM) accumulate
    that BatchNorm's backward reductions — sum(dy_eff), sum(dy_eff * xhat) — in its epilogue,
    so the BatchNorm backward skips its reduce pass over (dy, x).

    The BatchNorm's forward binds its saved tensors; the consumer's backward runs the
    GEMM with the BN-backward epilogue into the shared statistics workspace and sets
    ``ready``; the BatchNorm's backward then only finalizes and applies. Valid only when the
    linked consumer's dgrad output IS the whole gradient of the BatchNorm output (a single
    consumer, or the residual sum handed over through a :class:`GradLink`); otherwise the
    link stays unused and the BatchNorm reduces as usual.
    """

    __slots__ = ("x", "mask", "w32", "b32", "mean", "inv", "relu", "ready")

    def __init__(self):
        self.x = self.mask = self.w32 = self.b32 = self.mean = self.inv = None
        self.relu = False
        self.ready = False

    def bind(self, x, mask, w32, b32, mean, inv, relu):
        self.x, self.mask, self.w32, self.b32, self.mean, self.inv, self.relu = x, mask, w32, b32, mean, inv, relu
        self.ready = False

    @property
    def bound(self) -> bool:
        return self.x is not None

    @property
    def relu_mode(self) -> int:
        """0: no ReLU; 2: mask recomputed from x; 3: saved 1-bit mask."""
        return 0 if not self.relu else (3 if self.mask is not None else 2)

    def release(self):
        self.x = self.mask = self.w32 = self.b32 = self.mean = self.inv = None
        self.ready = False


def bn_counter(bn):
    """(momentum, counter) for a training-mode BatchNorm module: the ``num_batches_tracked``
    tensor the finalize kernel increments (no launch of its own), or None when nothing is
    tracked / the cumulative average (momentum None) needs the host-side count now."""
    if not (bn.training and bn.track_running_stats):
        return (0.1 if bn.momentum is None else bn.momentum), None
    if bn.momentum is None:
        bn.num_batches_tracked.add_(1)
        return 1.0 / float(bn.num_batches_tracked), None
    return bn.momentum, bn.num_batches_tracked


class _FusedBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, momentum, eps, relu, link=None,
                nbt=None, bnlink=None):
        C = _ext.get(required=True)
        x = _nhwc(x)
        res = _nhwc(residual) if residual is not None else None
        rows, ch = _rows_c(x)
        y = torch.empty_like(x)
        w32 = weight.float() if weight is not None else None
        b32 = bias.float() if bias is not None else None
        save_mean = torch.empty(ch, device=x.device, dtype=torch.float32)
        save_inv = torch.empty(ch, device=x.device, dtype=torch.float32)
        ws = _workspace(x)
        # ReLU after a residual add: keep a 1-bit mask (1/16 of y's bytes) for the backward
        mask = torch.empty(x.numel() // 8, device=x.device, dtype=torch.uint8) if (relu and res is not None) \
            else None
        stream = torch.cuda.current_stream(x.device).cuda_stream
        C.bn_fwd_train(x.data_ptr(), y.data_ptr(), res.data_ptr() if res is not None else 0,
                       w32.data_ptr() if w32 is not None else 0, b32.data_ptr() if b32 is not None else 0,
                       running_mean.data_ptr() if running_mean is not None else 0,
                       running_var.data_ptr() if running_var is not None else 0,
                       save_mean.data_ptr(), save_inv.data_ptr(), ws.data_ptr(), rows, ch, float(momentum),
                       float(eps), int(relu), mask.data_ptr() if mask is not None else 0, DTYPE_CODE[x.dtype], stream,
                       nbt.data_ptr() if nbt is not None else 0)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.link = link if residual is not None else None
        ctx.wdtype = weight.dtype if weight is not None else None
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        # Without a residual the ReLU mask is recomputed from x in the backward
        # kernels (bit-identical to the forward); with one, the 1-bit mask is used.
        # Either way y is neither saved nor re-read.
        ctx.save_for_backward(x, mask, w32, b32, save_mean, save_inv)
        ctx.bnlink = bnlink
        if bnlink is not None:
            bnlink.bind(x, mask, w32 if w32 is not None else torch.ones(ch, device=x.device),
                        b32 if b32 is not None else torch.zeros(ch, device=x.device), save_mean, save_inv, relu)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.get(required=True)
        x, mask, w32, b32, save_mean, save_inv = ctx.saved_tensors
        dy = _nhwc(dy)
        # the producer of dy already accumulated this BN's reductions into the workspace
        stats_ready = ctx.bnlink is not None and ctx.bnlink.ready
        rows, ch = _rows_c(x)
        dx = torch.empty_like(x)
        # a masked GradLink takes (dy, mask) instead of dres = dy * mask: one write pass less
        hand_masked = ctx.link is not None and ctx.link.masked and mask is not None and ctx.relu
        dres = torch.empty_like(x) if (ctx.has_res and not hand_masked) else None
        # the finalize kernel always produces both reductions (they feed dx)
        # fp32 parameters: straight into their DDP bucket slices when attached (graddst)
        dw, db = (_grad_out(p, ch, x) for p in ctx.params)
        ws = _link_workspace(x) if stats_ready else _workspace(x)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        C.bn_bwd(dy.data_ptr(), x.data_ptr(), 0, mask.data_ptr() if mask is not None else 0,
                 w32.data_ptr() if w32 is not None else 0, b32.data_ptr() if b32 is not None else 0,
                 save_mean.data_ptr(), save_inv.data_ptr(), dx.data_ptr(),
                 dres.data_ptr() if dres is not None else 0, dw.data_ptr(), db.data_ptr(), ws.data_ptr(), rows, ch,
                 int(ctx.relu), DTYPE_CODE[x.dtype], stream, int(stats_ready))
        if ctx.bnlink is not None:
            ctx.bnlink.release()
        if w32 is None:
            dw = None
        elif ctx.wdtype != torch.float32:
            dw = dw.to(ctx.wdtype)
        if not ctx.has_bias:
            db = None
        elif ctx.wdtype != torch.float32:
            db = db.to(ctx.wdtype)
        if ctx.link is not None:
            ctx.link.grad, dres = ((dy, mask) if hand_masked else dres), None
        return dx, dw, db, dres, None, None, None, None, None, None, None, None


def batch_norm_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu=False,
                         residual=None):
    """PyTorch composition with the same semantics (fp32 math)."""
    y = F.batch_norm(x.float(), running_mean, running_var, weight.float() if weight is not None else None,
                     bias.float() if bias is not None else None, training, momentum, eps)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = F.relu(y)
    return y.to(x.dtype)


def fused_batch_norm(x, weight, bias, running_mean, running_var, training=True, momentum=0.1, eps=1e-5,
                     relu=False, residual=None, link: GradLink | None = None,
                     num_batches_tracked: torch.Tensor | None = None, bnlink: BNStatsLink | None = None):
    """``link``: deliver the residual's gradient through a :class:`GradLink` instead of
    returning it to autograd (training with the fused kernels only; otherwise ignored).
    ``num_batches_tracked``: counter incremented once (inside the finalize kernel)."""
    if training and kernel_supported(x):
        return _FusedBN.apply(x, weight, bias, residual, running_mean, running_var, momentum, eps, relu, link,
                              num_batches_tracked, bnlink)
    if num_batches_tracked is not None and training:
        num_batches_tracked.add_(1)
    if (not training) and kernel_supported(x) and not torch.is_grad_enabled():
        C = _ext.get(required=True)
        x = _nhwc(x)
        rows, ch = _rows_c(x)
        y = torch.empty_like(x)
        res = _nhwc(residual) if residual is not None else None
        C.bn_fwd_infer(x.data_ptr(), y.data_ptr(), res.data_ptr() if res is not None else 0,
                       weight.float().data_ptr() if weight is not None else 0,
                       bias.float().data_ptr() if bias is not None else 0, running_mean.data_ptr(),
                       running_var.data_ptr(), rows, ch, float(eps), int(relu), DTYPE_CODE[x.dtype],
                       torch.cuda.current_stream(x.device).cuda_stream)
        return y
    return batch_norm_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu, residual)


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with optional fused ReLU / residual add (NHWC HIP kernels on GPU)."""

    def forward(self, x, relu: bool = False, residual: torch.Tensor | None = None, link: GradLink | None = None,
                bnlink: BNStatsLink | None = None):
        mom, nbt = bn_counter(self)
        use_batch = self.training or not self.track_running_stats
        return fused_batch_norm(x, self.weight, self.bias,
                                self.running_mean if self.track_running_stats else None,
                                self.running_var if self.track_running_stats else None,
                                use_batch, mom, self.eps, relu, residual, link, nbt, bnlink)
