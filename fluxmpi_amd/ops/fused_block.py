"""Producer/consumer fusion of 1x1 convolutions with BatchNorm for bottleneck blocks.

Built on the MFMA GEMM (``csrc/kernels/gemm.hip``) and the split fused-BN
kernels (``csrc/kernels/batchnorm.hip``). Per ResNet bottleneck:

=========================  ===================================================
op                         what disappears compared with conv -> BN -> ReLU
=========================  ===================================================
``conv1x1_stats``          the BatchNorm statistics pass over the conv output
                           (sums come from the GEMM epilogue)
``bn_relu_conv1x1``        the normalised activation: BN + ReLU are applied to
                           the GEMM's A operand while staging (forward) and to
                           the wgrad B operand (backward); never written to HBM
``bn_from_stats``          (consumer of the above) finalize + normalise pass only
``GradLink``               the residual-gradient add of the block input: the
                           BN backward hands ``dres`` to the conv1 dgrad GEMM,
                           which adds it in its epilogue
``conv1x1_hybrid``         MIOpen forward/wgrad, our dgrad (+ linked residual)
=========================  ===================================================

All three are autograd Functions; activations are bf16 NHWC (channels_last),
weights bf16, BatchNorm parameters / statistics fp32. Numerics: the BN affine
applied inside the GEMM is computed exactly like the fused-BN kernels'
(``scale = w * invstd``, ``shift = fma(-mean, scale, b)``), so ReLU masks
recomputed in the backward match the forward bit for bit.
"""
from __future__ import annotations

import torch

from . import _ext
from . import graddst
from .batchnorm import BNStatsLink, GradLink, SideGradLink, _dual_workspace, _link_workspace, _workspace, bn_counter  # noqa: F401 (links re-exported)
from . import gemm as G
from . import gemm_nt as _NT
from . import groupnorm as _GN
from .conv_choice import (_DGRAD_CHOICE, _DS_CHOICE, _FWD1_CHOICE, _FWD_CHOICE, _FWD_ENGINE, _S2_CHOICE,  # noqa: F401
                          _WG_CHOICE, FWD_ENGINES, choices_frozen, dump_choices, freeze_choices,
                          load_choice_lines, load_choices, no_measure as _no_measure, stats_choice,
                          time_us as _time_us, w256_ok as _w256_ok, w3n_configs, wgrad_best)
from .gemm import conv1x1_dgrad, conv1x1_wgrad, conv3x3_dgrad, conv3x3_fwd, gemm, note_filter
from .multi_tensor import DTYPE_CODE


# 3x3 / stride-1 convolutions of the bottlenecks: "ours" = forward (+ the next BatchNorm's
# statistics in the epilogue) and input gradient on the implicit-GEMM MFMA kernel, weight
# gradient on MIOpen; "dgrad" = only the input gradient ours; "miopen" = all MIOpen
CONV3X3 = "ours"
# 1x1 forward of the bottlenecks: "ours" = our GEMM + statistics epilogue where measured faster
# than MIOpen + the statistics pass; "miopen" = always MIOpen
CONV1X1 = "ours"
# downsample blocks: bn3 and the downsample branch's BatchNorm as one dual kernel pair
# (relu(bn3(c3) + bn_ds(c_ds)) without materialising bn_ds(c_ds); see dual_bn_relu)
DUAL_BN = True
# downsample 1x1 forward: "ours" = our GEMM (stride 2 gathers the even pixels in the A staging)
# with the downsample BatchNorm's sums in its epilogue where measured faster than MIOpen + the
# statistics pass (dual-BN blocks only); "force" = ours wherever supported; "miopen" = always MIOpen
DS_FWD = "ours"
# weight gradients of the downsample 1x1 and the stride-2 3x3 convolutions: MIOpen vs our split-K
# kernel (stride-2 B-row gather / implicit stride-2 im2col), measured per shape
DS_WGRAD = True
# stride-2 3x3 forward: our implicit GEMM (+ statistics epilogue) where measured faster (0: MIOpen)
S2_FWD = True


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return t.data_ptr() if t is not None else 0


def _nhwc2d(x: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] channels_last -> [N*H*W, C] view (copy if not channels_last)."""
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _empty_nhwc(n, c, h, w, like):
    return torch.empty(n, h, w, c, device=like.device, dtype=like.dtype).permute(0, 3, 1, 2)


def _grad_out(p, ch, like):
    """fp32 [ch] output for the gradient of BatchNorm parameter ``p``: its DDP bucket slice when
    one is attached (``graddst``, fp32 parameters), else a fresh tensor."""
    t = graddst.take(p, (ch,), torch.float32)
    return t if t is not None else torch.empty(ch, device=like.device, dtype=torch.float32)


def _fwd1x1_stats(x, weight, stats):
    """c = conv1x1(x, W) (NHWC) with the output's BatchNorm sums into ``stats``: on the 256x256
    persistent kernel (``gemm_nt``, statistics epilogue) where the shape qualifies (``gemm_nt.gemm_ok``:
    enough tiles and K), else on the LDS-DMA GEMM."""
    n, ci, h, w = x.shape
    co = weight.shape[0]
    c = _empty_nhwc(n, co, h, w, x)
    x2, w2 = _nhwc2d(x), weight.reshape(co, ci)
    if G.ENGINE != 1 and _NT.gemm_ok(n * h * w, co, ci, x2, w2):
        _NT.gemm_plain(x2, w2, _nhwc2d(c), stats)
    else:
        gemm(x2, w2, c, M=n * h * w, N=co, K=ci, lda=ci, ldb=ci, ldc=co, a_kmajor=True, b_kmajor=True, mode=1,
             stats=stats)
    return c


def _bn_bwd(dy, x, mask, w32, b32, mean, inv, relu, has_res, stats_ready=False, params=(None, None)):
    """Shared fused-BN backward; returns (dx, dres, dw, db) (fp32 dw/db; ``params`` = the
    (weight, bias) leaves whose bucket slices may receive them)."""
    C = _ext.get(required=True)
    rows, ch = x.numel() // x.shape[1], x.shape[1]
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if has_res else None
    dw = _grad_out(params[0], ch, x)
    db = _grad_out(params[1], ch, x)
    ws = _link_workspace(x) if stats_ready else _workspace(x)
    C.bn_bwd(dy.data_ptr(), x.data_ptr(), 0, _p(mask), _p(w32), _p(b32), mean.data_ptr(), inv.data_ptr(),
             dx.data_ptr(), _p(dres), dw.data_ptr(), db.data_ptr(), ws.data_ptr(), rows, ch, int(relu),
             DTYPE_CODE[x.dtype], _stream(x), int(stats_ready))
    return dx, dres, dw, db


class _Conv1x1Stats(torch.autograd.Function):
    """c = conv1x1(x, W); the output's per-channel sum/sumsq go to the BN workspace."""

    @staticmethod
    def forward(ctx, x, weight, link=None, bnlink=None):
        x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
        ctx.link, ctx.bnlink = link, bnlink
        note_filter(weight)
        c = _fwd1x1_stats(x, weight, _workspace(x))
        ctx.save_for_backward(x, weight)
        return c

    @staticmethod
    def backward(ctx, dc):
        x, weight = ctx.saved_tensors
        co, ci = weight.shape[0], weight.shape[1]
        dc2 = _nhwc2d(dc)
        # weight gradient first, on the side stream: it overlaps the input-gradient chain
        with graddst.into(weight):  # into the DDP bucket slice when one is attached
            dw = conv1x1_wgrad(dc2, _nhwc2d(x), out_dtype=weight.dtype).view_as(weight)
        dx = _dgrad_nhwc(dc2, weight, x, ctx.link, ctx.bnlink) if ctx.needs_input_grad[0] else None
        return dx, dw, None, None


class Stride2Grad:
    """The input gradient of a stride-2 1x1 convolution in compact form ([N, C, ceil(H/2),
    ceil(W/2)]: only the even positions of the full-resolution gradient are nonzero), as handed
    through a :class:`SideGradLink`; the consumer's dgrad epilogue adds it at even (h, w)."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def expand(self, shape):
        n, c, h, w = shape
        full = _empty_nhwc(n, c, h, w, self.t).zero_()
        full[:, :, ::2, ::2] = self.t
        return full


def _dgrad_nhwc(dc2, weight, x, link, bnlink=None):
    """dX (NHWC, x's shape) = dC @ W [+ the residual gradient delivered through ``link``]; with a
    bound ``bnlink`` the epilogue also accumulates the backward reductions of the BatchNorm
    that produced x (whose output gradient dX is), so that BatchNorm skips its reduce pass."""
    co, ci = weight.shape[0], weight.shape[1]
    n, _, h, w = x.shape
    dx = _empty_nhwc(n, ci, h, w, x)
    res = res_mask = res_sub = None
    if link is not None:
        g = link.take()  # SideGradLink: None if its producer has not run (it then returns its own)
        if isinstance(g, tuple):  # masked GradLink: (dy, 1-bit ReLU mask), masked in the epilogue
            res, res_mask = _nhwc2d(g[0]), g[1]
        elif isinstance(g, Stride2Grad):  # compact gradient of a stride-2 1x1 conv's input
            res, res_sub = _nhwc2d(g.t), (h, w)
        elif g is not None:
            res = _nhwc2d(g)
    bn = stats = None
    if bnlink is not None and bnlink.bound and bnlink.x.shape == x.shape and \
            bnlink.x.is_contiguous(memory_format=torch.channels_last):
        bn = (_nhwc2d(bnlink.x), bnlink.w32, bnlink.b32, bnlink.mean, bnlink.inv, bnlink.mask, bnlink.relu_mode)
        stats = _link_workspace(dx)
    conv1x1_dgrad(dc2, weight.reshape(co, ci), residual=res, out=_nhwc2d(dx), bn_bwd=bn, stats=stats, w4d=weight,
                  residual_mask=res_mask, residual_sub=res_sub)
    if bn is not None:
        bnlink.ready = True
    return dx


class _Conv1x1Hybrid(torch.autograd.Function):
    """1x1 convolution: forward and weight gradient on MIOpen (fastest there), input
    gradient on our MFMA GEMM (faster than MIOpen's on every ResNet-50 shape measured)
    with the block's residual gradient added in its epilogue (``link``)."""

    @staticmethod
    def forward(ctx, x, weight, link=None, bnlink=None, ours_stats=False):
        x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
        ctx.link, ctx.bnlink = link, bnlink
        note_filter(weight)
        ctx.save_for_backward(x, weight)
        if ours_stats:
            # our GEMM, the next BatchNorm's statistics accumulated in its epilogue
            return _fwd1x1_stats(x, weight, _workspace(x))
        return torch.nn.functional.conv2d(x, weight)

    @staticmethod
    def backward(ctx, dc):
        x, weight = ctx.saved_tensors
        if not dc.is_contiguous(memory_format=torch.channels_last):
            dc = dc.contiguous(memory_format=torch.channels_last)
        dw = None
        if ctx.needs_input_grad[1]:
            co, ci = weight.shape[0], weight.shape[1]
            impls = {
                "miopen": lambda: torch.ops.aten.convolution_backward(dc, x, weight, None, [1, 1], [0, 0], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False])[1],
                "ours": lambda: G.conv1x1_wgrad_v2(_nhwc2d(dc), _nhwc2d(x), out_dtype=weight.dtype).view(co, ci, 1, 1)}
            if _w256_ok(co, ci, dc):
                from .linear import weight_grad
                impls["w256"] = lambda: weight_grad(_nhwc2d(dc), _nhwc2d(x), weight.dtype).view(co, ci, 1, 1)
            dw = wgrad_best(("1x1", tuple(x.shape), co), impls, param=weight)
        dx = _dgrad_nhwc(_nhwc2d(dc), weight, x, ctx.link, ctx.bnlink) if ctx.needs_input_grad[0] else None
        return dx, dw, None, None, None


def _ds_fwd_ours(x, weight, stride, stats):
    """The downsample convolution on our GEMM (stride 2: A rows gathered from the even pixels,
    no strided copy), its BatchNorm's per-channel sums into ``stats``."""
    n, ci, h, w = x.shape
    co = weight.shape[0]
    ho, wo = (h + stride - 1) // stride, (w + stride - 1) // stride
    c = _empty_nhwc(n, co, ho, wo, x)
    gemm(_nhwc2d(x), weight.reshape(co, ci), c, M=n * ho * wo, N=co, K=ci, lda=ci, ldb=ci, ldc=co, mode=1,
         stats=stats, a_sub=(h, w) if stride == 2 else None)
    return c


def ds_forward_supported(x, weight, stride) -> bool:
    return (DS_FWD in ("ours", "force") and G.ENGINE != 1 and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and weight.dtype == torch.bfloat16 and stride in (1, 2) and x.shape[1] % 8 == 0
            and weight.shape[0] % 8 == 0 and x.numel() // x.shape[1] < 2 ** 31)


def ds_forward_is_ours(x, weight, stride) -> bool:
    """Per-shape choice of the downsample forward, measured once: our GEMM with the statistics
    epilogue vs MIOpen plus the statistics pass its BatchNorm then needs (one read of the output
    at 5 TB/s)."""
    if not ds_forward_supported(x, weight, stride):
        return False
    if DS_FWD == "force":
        return True
    def make():
        xs, w = x.detach().contiguous(memory_format=torch.channels_last), weight.detach()
        n, _, h, wd = x.shape
        ws = torch.zeros_like(_workspace(xs))
        return (lambda: _ds_fwd_ours(xs, w, stride, ws), lambda: torch.nn.functional.conv2d(xs, w, None, stride),
                n * ((h + stride - 1) // stride) * ((wd + stride - 1) // stride) * w.shape[0] * x.element_size())
    return stats_choice(_DS_CHOICE, (tuple(x.shape), weight.shape[0], stride), make)


class _Conv1x1Downsample(torch.autograd.Function):
    """The downsample 1x1 convolution (stride 1 or 2) of a ResNet block: forward on MIOpen, or
    (``stats``) on our GEMM with its BatchNorm's sums left pending in ``stats`` (the dual BN
    consumes them); weight gradient on MIOpen. Its input gradient (our dgrad GEMM; at stride 2
    over the output pixels only, in the compact :class:`Stride2Grad` form) is handed to the
    block's conv1 through a :class:`SideGradLink`, whose dgrad epilogue adds it: no separate add
    kernel over the block input's gradient, and at stride 2 no zero-filled full-resolution
    gradient either."""

    @staticmethod
    def forward(ctx, x, weight, stride, link, stats=None):
        x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
        ctx.stride, ctx.link = stride, link
        note_filter(weight)
        ctx.save_for_backward(x, weight)
        if stats is not None:
            return _ds_fwd_ours(x, weight, stride, stats)
        return torch.nn.functional.conv2d(x, weight, None, stride)

    @staticmethod
    def backward(ctx, dc):
        x, weight = ctx.saved_tensors
        if not dc.is_contiguous(memory_format=torch.channels_last):
            dc = dc.contiguous(memory_format=torch.channels_last)
        s = ctx.stride
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if s == 1 and need_x:
            dx = _dgrad_nhwc(_nhwc2d(dc), weight, x, None)
        elif s == 2 and need_x and ctx.link is not None and G.ENGINE != 1 and x.shape[1] % 8 == 0:
            # compact: the GEMM over the strided output pixels only; conv1's dgrad epilogue adds it
            # at the even positions (no zero-filled full-resolution gradient is written or read)
            n, co, ho, wo = dc.shape
            ci = weight.shape[1]
            dxc = _empty_nhwc(n, ci, ho, wo, dc)
            conv1x1_dgrad(_nhwc2d(dc), weight.reshape(co, ci), out=_nhwc2d(dxc), w4d=weight)
            if ctx.link.offer(Stride2Grad(dxc)):
                dxc = None
                need_x = False  # delivered
            else:
                dx = Stride2Grad(dxc).expand(x.shape)
        if need_w and not (need_x and dx is None):
            dw = _ds_wgrad(dc, x, weight, s)
        elif need_w or (need_x and dx is None):
            dx_m, dw = torch.ops.aten.convolution_backward(dc, x, weight, None, [s, s], [0, 0], [1, 1], False,
                                                           [0, 0], 1, [need_x and dx is None, need_w, False])[:2]
            dx = dx if dx is not None else dx_m
        if dx is not None and ctx.link is not None and ctx.link.offer(dx):
            dx = None  # delivered to conv1's dgrad epilogue
        return dx, dw, None, None, None


def _ds_wgrad(dc, x, weight, s):
    """The downsample convolution's weight gradient: the fastest (measured once per shape) of
    MIOpen and our split-K kernel (stride 2: B rows gathered from the even pixels)."""
    co, ci = weight.shape[0], weight.shape[1]
    impls = {"miopen": lambda: torch.ops.aten.convolution_backward(
        dc, x, weight, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])[1]}
    if DS_WGRAD and dc.dtype == torch.bfloat16 and ci % 8 == 0 and co % 8 == 0 and G.ENGINE != 1:
        if s == 1:
            impls["ours"] = lambda: G.conv1x1_wgrad_v2(_nhwc2d(dc), _nhwc2d(x), out_dtype=weight.dtype).view(
                co, ci, 1, 1)
            if _w256_ok(co, ci, dc):
                from .linear import weight_grad
                impls["w256"] = lambda: weight_grad(_nhwc2d(dc), _nhwc2d(x), weight.dtype).view(co, ci, 1, 1)
        elif s == 2:
            impls["ours"] = lambda: G.conv1x1_wgrad_s2(_nhwc2d(dc), x, out_dtype=weight.dtype).view(co, ci, 1, 1)
    if "ours" not in impls:
        return impls["miopen"]()
    return wgrad_best(("ds", tuple(x.shape), co, s), impls, param=weight)


def conv1x1_downsample(x, weight, stride, link=None, ours_stats=False):
    """``ours_stats`` (see :func:`ds_forward_is_ours`): forward on our GEMM with the output's
    BatchNorm sums pending in the dual workspace, for ``dual_bn_relu(..., ds_stats_ready=True)``."""
    return _Conv1x1Downsample.apply(x, weight, stride, link, _dual_workspace(x) if ours_stats else None)


class _BNFromStats(torch.autograd.Function):
    """BatchNorm(+residual)(+ReLU) whose batch statistics are already in the workspace
    (``stats_ready``) or are computed by the stats pass here."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, momentum, eps, relu, stats_ready,
                link=None, nbt=None, bnlink=None):
        C = _ext.get(required=True)
        ch = x.shape[1]
        rows = x.numel() // ch
        w32 = weight.float()
        b32 = bias.float()
        mean = torch.empty(ch, device=x.device, dtype=torch.float32)
        inv = torch.empty(ch, device=x.device, dtype=torch.float32)
        ws = _workspace(x)
        C.bn_stats_finalize(x.data_ptr(), w32.data_ptr(), b32.data_ptr(), _p(running_mean), _p(running_var),
                            mean.data_ptr(), inv.data_ptr(), 0, 0, ws.data_ptr(), rows, ch, float(momentum),
                            float(eps), int(stats_ready), DTYPE_CODE[x.dtype], _stream(x), _p(nbt))
        res = None
        if residual is not None:
            res = residual if residual.is_contiguous(memory_format=torch.channels_last) else \
                residual.contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(x)
        mask = torch.empty(x.numel() // 8, device=x.device, dtype=torch.uint8) if (relu and res is not None) \
            else None
        C.bn_apply(x.data_ptr(), y.data_ptr(), _p(res), w32.data_ptr(), b32.data_ptr(), mean.data_ptr(),
                   inv.data_ptr(), rows, ch, int(relu), _p(mask), DTYPE_CODE[x.dtype], _stream(x))
        ctx.relu, ctx.has_res, ctx.wdtype = relu, residual is not None, weight.dtype
        ctx.params = (weight, bias)
        ctx.link = link if residual is not None else None
        ctx.bnlink = bnlink
        if bnlink is not None:
            bnlink.bind(x, mask, w32, b32, mean, inv, relu)
        ctx.save_for_backward(x, mask, w32, b32, mean, inv)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, w32, b32, mean, inv = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        ready = ctx.bnlink is not None and ctx.bnlink.ready
        # a masked GradLink takes (dy, mask) instead of dres = dy * mask (one write pass less)
        hand_masked = ctx.link is not None and ctx.link.masked and mask is not None and ctx.relu
        dx, dres, dw, db = _bn_bwd(dy, x, mask, w32, b32, mean, inv, ctx.relu, ctx.has_res and not hand_masked,
                                   ready, ctx.params)
        if ctx.bnlink is not None:
            ctx.bnlink.release()
        if ctx.link is not None:
            ctx.link.grad, dres = ((dy, mask) if hand_masked else dres), None
        return dx, dw.to(ctx.wdtype), db.to(ctx.wdtype), dres, None, None, None, None, None, None, None, None, None


class _DualBN(torch.autograd.Function):
    """out = relu(bn3(c3) + bn_ds(c_ds)) for a ResNet downsample block, without materialising the
    downsample branch's output bn_ds(c_ds). Forward: bn3's statistics (pending from the conv3
    GEMM epilogue when ``stats_ready``, else a stats pass), bn_ds's stats pass, one apply pass
    reading (c3, c_ds). Backward: dy_eff = dy * relu_mask is the output gradient of BOTH
    BatchNorms, so one reduce pass over (dy, mask, c3, c_ds) produces both BatchNorms' sums
    and one pass writes both input gradients: versus two separate BatchNorms, the identity is
    neither written nor read forward, and dres is neither written nor read twice backward
    (~10 B/element saved on a block's largest activations)."""

    @staticmethod
    def forward(ctx, c3, w, b, rm, rv, mom, eps, nbt, stats_ready, cds, w2, b2, rm2, rv2, mom2, eps2, nbt2,
                ds_ready=False):
        C = _ext.get(required=True)
        cl = torch.channels_last
        c3 = c3 if c3.is_contiguous(memory_format=cl) else c3.contiguous(memory_format=cl)
        cds = cds if cds.is_contiguous(memory_format=cl) else cds.contiguous(memory_format=cl)
        ch = c3.shape[1]
        rows = c3.numel() // ch
        f32 = dict(device=c3.device, dtype=torch.float32)
        w32, b32, w232, b232 = w.float(), b.float(), w2.float(), b2.float()
        mean, inv, mean2, inv2 = (torch.empty(ch, **f32) for _ in range(4))
        ws, code, st = _workspace(c3), DTYPE_CODE[c3.dtype], _stream(c3)
        # bn3 first: its sums may be pending in the workspace (conv3's GEMM epilogue)
        C.bn_stats_finalize(c3.data_ptr(), w32.data_ptr(), b32.data_ptr(), _p(rm), _p(rv), mean.data_ptr(),
                            inv.data_ptr(), 0, 0, ws.data_ptr(), rows, ch, float(mom), float(eps), int(stats_ready),
                            code, st, _p(nbt))
        # bn_ds: its sums pending in the dual workspace (the downsample GEMM's epilogue), or a stats pass
        ws2 = _dual_workspace(c3) if ds_ready else ws
        C.bn_stats_finalize(cds.data_ptr(), w232.data_ptr(), b232.data_ptr(), _p(rm2), _p(rv2), mean2.data_ptr(),
                            inv2.data_ptr(), 0, 0, ws2.data_ptr(), rows, ch, float(mom2), float(eps2), int(ds_ready),
                            code, st, _p(nbt2))
        y = torch.empty_like(c3)
        mask = torch.empty(c3.numel() // 8, device=c3.device, dtype=torch.uint8)
        C.bn_apply_dual(c3.data_ptr(), cds.data_ptr(), y.data_ptr(), w32.data_ptr(), b32.data_ptr(), mean.data_ptr(),
                        inv.data_ptr(), w232.data_ptr(), b232.data_ptr(), mean2.data_ptr(), inv2.data_ptr(), rows, ch,
                        mask.data_ptr(), code, st)
        ctx.wdtypes = (w.dtype, w2.dtype)
        ctx.params = (w, b, w2, b2)
        ctx.save_for_backward(c3, cds, mask, w32, mean, inv, w232, mean2, inv2)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.get(required=True)
        c3, cds, mask, w32, mean, inv, w232, mean2, inv2 = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        ch = c3.shape[1]
        rows = c3.numel() // ch
        dx, dx2 = torch.empty_like(c3), torch.empty_like(cds)
        dw, db, dw2, db2 = (_grad_out(p, ch, c3) for p in ctx.params)
        C.bn_bwd_dual(dy.data_ptr(), mask.data_ptr(), c3.data_ptr(), cds.data_ptr(), w32.data_ptr(), mean.data_ptr(),
                      inv.data_ptr(), w232.data_ptr(), mean2.data_ptr(), inv2.data_ptr(), dx.data_ptr(),
                      dx2.data_ptr(), dw.data_ptr(), db.data_ptr(), dw2.data_ptr(), db2.data_ptr(),
                      _workspace(c3).data_ptr(), _dual_workspace(c3).data_ptr(), rows, ch, DTYPE_CODE[c3.dtype],
                      _stream(c3))
        t1, t2 = ctx.wdtypes
        return (dx, dw.to(t1), db.to(t1), None, None, None, None, None, None,
                dx2, dw2.to(t2), db2.to(t2), None, None, None, None, None, None)


def dual_bn_supported(c, bn, bn_ds) -> bool:
    """``dual_bn_relu`` applies: fused training-mode affine BatchNorms with running statistics,
    channels a power of two <= 2048 (C/8 divides the 256-lane workgroup)."""
    from .batchnorm import FusedBatchNorm2d, kernel_supported
    ch = c.shape[1]
    return (DUAL_BN and kernel_supported(c) and c.dim() == 4 and (ch & (ch - 1)) == 0
            and all(isinstance(m, FusedBatchNorm2d) and m.training and m.affine and m.track_running_stats
                    for m in (bn, bn_ds)))


def dual_bn_relu(c3, bn, cds, bn_ds, stats_ready=False, ds_stats_ready=False):
    """relu(bn(c3) + bn_ds(cds)) (training); ``stats_ready``: bn's sums are pending in the
    workspace from the GEMM that produced c3; ``ds_stats_ready``: bn_ds's sums are pending in the
    dual workspace (``conv1x1_downsample(..., ours_stats=True)``)."""
    mom, nbt = bn_counter(bn)
    mom2, nbt2 = bn_counter(bn_ds)
    return _DualBN.apply(c3, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps, nbt, stats_ready,
                         cds, bn_ds.weight, bn_ds.bias, bn_ds.running_mean, bn_ds.running_var, mom2, bn_ds.eps, nbt2,
                         ds_stats_ready)


def dual_bn_ok(x, ch, bn, bn_ds) -> bool:
    """:func:`dual_bn_supported` for the output (``ch`` channels, x's dtype/device) of a
    convolution of ``x``, decided before running it."""
    from .batchnorm import FusedBatchNorm2d
    return (DUAL_BN and x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and x.dim() == 4
            and ch % 8 == 0 and 8 <= ch <= 2048 and (ch & (ch - 1)) == 0
            and all(isinstance(m, FusedBatchNorm2d) and m.training and m.affine and m.track_running_stats
                    for m in (bn, bn_ds)))


class _BNReluConv1x1(torch.autograd.Function):
    """c3 = conv1x1(relu(BN(c2)), W) without materialising relu(BN(c2)); c3's statistics
    go to the workspace (consumed by the next ``bn_from_stats``)."""

    @staticmethod
    def forward(ctx, c2, bn_weight, bn_bias, running_mean, running_var, weight, momentum, eps, nbt=None,
                stats_ready=False):
        C = _ext.get(required=True)
        if not c2.is_contiguous(memory_format=torch.channels_last):
            c2 = c2.contiguous(memory_format=torch.channels_last)
        n, ch, h, w = c2.shape
        rows = n * h * w
        w32, b32 = bn_weight.float(), bn_bias.float()
        mean = torch.empty(ch, device=c2.device, dtype=torch.float32)
        inv = torch.empty_like(mean)
        scale = torch.empty_like(mean)
        shift = torch.empty_like(mean)
        ws = _workspace(c2)
        C.bn_stats_finalize(c2.data_ptr(), w32.data_ptr(), b32.data_ptr(), _p(running_mean), _p(running_var),
                            mean.data_ptr(), inv.data_ptr(), scale.data_ptr(), shift.data_ptr(), ws.data_ptr(),
                            rows, ch, float(momentum), float(eps), int(stats_ready), DTYPE_CODE[c2.dtype], _stream(c2),
                            _p(nbt))
        co = weight.shape[0]
        c3 = _empty_nhwc(n, co, h, w, c2)
        gemm(_nhwc2d(c2), weight.reshape(co, ch), c3, M=rows, N=co, K=ch, lda=ch, ldb=ch, ldc=co, a_kmajor=True,
             b_kmajor=True, mode=1, stats=ws, a_affine=(scale, shift))
        ctx.bn_wdtype = bn_weight.dtype
        ctx.params = (bn_weight, bn_bias)  # the leaves: their gradients' bucket slices (graddst)
        ctx.save_for_backward(c2, w32, b32, mean, inv, scale, shift, weight)
        return c3

    @staticmethod
    def backward(ctx, dc3):
        c2, w32, b32, mean, inv, scale, shift, weight = ctx.saved_tensors
        n, ch, h, w = c2.shape
        co = weight.shape[0]
        dc3_2d = _nhwc2d(dc3)
        c2_2d = _nhwc2d(c2)
        # dW = dc3^T @ relu(bn(c2))  — the activation is rebuilt on the fly in the B-operand load
        # (side stream: overlaps the input-gradient chain below)
        with graddst.into(weight):
            dw = conv1x1_wgrad(dc3_2d, c2_2d, in_affine=(scale, shift), out_dtype=weight.dtype).view_as(weight)
        # d(relu(bn(c2))) = dc3 @ W with the BN-backward reductions (ReLU mask recomputed from c2)
        # accumulated in the same GEMM's epilogue, then the BN backward without its reduce pass
        # (w4d: the LDS-DMA kernel on the cached W^T, whose epilogue has the BN-backward reductions)
        da = conv1x1_dgrad(dc3_2d, weight.reshape(co, ch), bn_bwd=(c2_2d, w32, b32, mean, inv, None, 2),
                           stats=_link_workspace(c2), w4d=weight).view(n, h, w, ch).permute(0, 3, 1, 2)
        dc2, _, dbw, dbb = _bn_bwd(da, c2, None, w32, b32, mean, inv, True, False, stats_ready=True,
                                   params=ctx.params)
        return dc2, dbw.to(ctx.bn_wdtype), dbb.to(ctx.bn_wdtype), None, None, dw, None, None, None, None


class _Conv3x3(torch.autograd.Function):
    """3x3 / stride 1 / pad 1 convolution: implicit-GEMM forward (optionally with the next
    BatchNorm's statistics accumulated in its epilogue) and input gradient on the LDS-DMA
    MFMA kernel; weight gradient on MIOpen."""

    @staticmethod
    def forward(ctx, x, weight, fwd_ours, with_stats, bnlink=None, gradlink=None):
        x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
        ctx.bnlink = bnlink
        ctx.gradlink = gradlink
        note_filter(weight)
        if fwd_ours:
            y = conv3x3_fwd(x, weight, stats=_workspace(x) if with_stats else None,
                            engine=_FWD_ENGINE.get((tuple(x.shape), weight.shape[0])))
        else:
            y = torch.nn.functional.conv2d(x, weight, None, 1, 1)
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dw = None
        # (inside groupnorm.skip_param_grads — the DEQ adjoint's VJPs w.r.t. activations only — the
        # filter gradient is not wanted although needs_input_grad, fixed at forward time, says so)
        if ctx.needs_input_grad[1] and not _GN._SKIP_PARAM_GRADS:
            impls = {
                "miopen": lambda: torch.ops.aten.convolution_backward(dy, x, weight, None, [1, 1], [1, 1], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False])[1],
                "ours": lambda: G.conv3x3_wgrad(dy, x)}
            if x.dtype == torch.bfloat16 and G.wgrad3x3n_ok(tuple(x.shape), weight.shape[0]):
                impls["w3n"] = lambda cfg: G.conv3x3_wgrad_n(dy, x, *cfg)  # narrow channels: rows staged once
                impls["w3n_cfgs"] = w3n_configs(x.shape[1])
            dw = wgrad_best(("3x3", tuple(x.shape), weight.shape[0]), impls, param=weight)
        dx = None
        if ctx.needs_input_grad[0]:
            bl = ctx.bnlink
            bn = stats = None
            if bl is not None and bl.bound and bl.x.shape == x.shape and \
                    bl.x.is_contiguous(memory_format=torch.channels_last) and G.ENGINE != 1:
                # the epilogue reduces the backward statistics of the BatchNorm that produced x
                bn = (_nhwc2d(bl.x), bl.w32, bl.b32, bl.mean, bl.inv, bl.mask, bl.relu_mode)
                stats = _link_workspace(x)
            # gradlink: x's other consumer deposited its gradient of x (GroupNorm / BatchNorm backward
            # ran first: autograd orders it by data dependency); added in the dgrad epilogue
            res = ctx.gradlink.take() if ctx.gradlink is not None else None
            if bn is None and not _dgrad_is_ours(dy, weight, x.shape):
                dx = torch.ops.aten.convolution_backward(dy, x, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0],
                                                         1, [True, False, False])[0]
                if res is not None:
                    dx = dx + res
            elif res is not None and bn is not None:
                dx = conv3x3_dgrad(dy, weight, bn_bwd=bn, stats=stats) + res
            else:
                dx = conv3x3_dgrad(dy, weight, bn_bwd=bn, stats=stats, residual=res)
            if bn is not None:
                bl.ready = True
        elif ctx.gradlink is not None:
            ctx.gradlink.grad = None
        return dx, dw, None, None, None, None


def _dgrad_is_ours(dy, weight, x_shape) -> bool:
    """Input gradient on our implicit GEMM, or MIOpen. Channel counts that are multiples of 32
    (ResNet-50) always take ours; narrower ones (e.g. the 48-channel DEQ cell, whose K tiles
    straddle filter taps) are measured once per shape, like the forward."""
    if weight.shape[0] % 32 == 0:
        return True
    key = (tuple(x_shape), weight.shape[0])
    hit = _DGRAD_CHOICE.get(key)
    if hit is not None:
        return hit
    if _no_measure():
        return True
    with torch.no_grad():
        d = dy.detach()
        w = weight.detach()
        xe = torch.empty(x_shape, device=dy.device, dtype=dy.dtype).contiguous(memory_format=torch.channels_last)
        ours = _time_us(lambda: conv3x3_dgrad(d, w))
        theirs = _time_us(lambda: torch.ops.aten.convolution_backward(d, xe, w, None, [1, 1], [1, 1], [1, 1], False,
                                                                      [0, 0], 1, [True, False, False]))
    _DGRAD_CHOICE[key] = ours <= theirs
    return _DGRAD_CHOICE[key]


class _Conv3x3S2(torch.autograd.Function):
    """3x3 / stride 2 / pad 1 convolution (the first conv2 of ResNet stages 2-4). Forward: MIOpen,
    or (``with_stats``) our implicit GEMM over the output pixels with the next BatchNorm's sums in
    its epilogue; input gradient on the four parity-class implicit GEMMs (``gemm.conv3x3_s2_dgrad``,
    even input sizes; MIOpen otherwise); weight gradient measured per shape between MIOpen and
    our split-K kernel over the stride-2 implicit im2col (``gemm.conv3x3_wgrad_s2``)."""

    @staticmethod
    def forward(ctx, x, weight, with_stats=False):
        x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
        ctx.save_for_backward(x, weight)
        if G.S2_DGRAD:
            note_filter(weight)  # the input gradient reads the batched transposed-filter cache
        if with_stats:
            return G.conv3x3_s2_fwd(x, weight, stats=_workspace(x))
        return torch.nn.functional.conv2d(x, weight, None, 2, 1)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = wgrad_best(("3x3s2", tuple(x.shape), weight.shape[0]), {
                "miopen": lambda: torch.ops.aten.convolution_backward(dy, x, weight, None, [2, 2], [1, 1], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False])[1],
                "ours": lambda: G.conv3x3_wgrad_s2(dy, x)}, param=weight)
        if ctx.needs_input_grad[0]:
            if G.s2_dgrad_ok(dy, weight, x.shape):
                dx = G.conv3x3_s2_dgrad(dy, weight, x.shape)  # four parity-class implicit GEMMs
            else:
                dx = torch.ops.aten.convolution_backward(dy, x, weight, None, [2, 2], [1, 1], [1, 1], False, [0, 0],
                                                         1, [True, False, False])[0]
        return dx, dw, None


def conv3x3_s2_supported(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (DS_WGRAD and G.ENGINE != 1 and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 8 == 0 and conv.out_channels % 8 == 0 and conv.weight.dtype == torch.bfloat16
            and x.numel() // x.shape[1] < 2 ** 31)


def conv3x3_s2_forward_is_ours(x, weight) -> bool:
    """Per-shape choice of the stride-2 3x3 forward, measured once: our implicit GEMM with the
    statistics epilogue vs MIOpen plus the statistics pass (one read of the output at 5 TB/s)."""
    if CONV3X3 != "ours" or not S2_FWD or x.shape[1] % 32 != 0:
        return False
    def make():
        xs, w = x.detach().contiguous(memory_format=torch.channels_last), weight.detach()
        n, _, h, wd = x.shape
        ws = torch.zeros_like(_workspace(xs))
        return (lambda: G.conv3x3_s2_fwd(xs, w, stats=ws), lambda: torch.nn.functional.conv2d(xs, w, None, 2, 1),
                n * ((h + 1) // 2) * ((wd + 1) // 2) * w.shape[0] * x.element_size())
    return stats_choice(_S2_CHOICE, (tuple(x.shape), weight.shape[0]), make)


def conv3x3_s2(x, weight, with_stats=False):
    """``with_stats``: our forward, the output's BatchNorm sums pending in the workspace (consume
    with ``bn_from_stats(..., stats_ready=True)``); decide with :func:`conv3x3_s2_forward_is_ours`."""
    return _Conv3x3S2.apply(x, weight, with_stats)


def conv3x3_supported(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (CONV3X3 in ("ours", "dgrad") and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 8 == 0 and conv.out_channels % 8 == 0 and conv.weight.dtype == torch.bfloat16
            and x.numel() // x.shape[1] < 2 ** 31)


def conv3x3_forward_is_ours(x, weight) -> bool:
    """Per-shape choice of the 3x3 forward, measured once (like cudnn.benchmark): our implicit
    GEMM with the statistics epilogue vs MIOpen plus the separate statistics pass it then needs
    (priced at one read of the output at 5 TB/s). Wave quantization makes some shapes (e.g.
    ResNet-50's 14x14x256 at batch 256: 1.5 rounds of 128x128 tiles) slower on our kernel."""
    if CONV3X3 != "ours":
        return False
    key = (tuple(x.shape), weight.shape[0])
    hit = _FWD_CHOICE.get(key)
    if hit is not None:
        return hit
    if _no_measure():
        return True
    with torch.no_grad():
        xs = x.detach().contiguous(memory_format=torch.channels_last)
        w = weight.detach()
        ws = torch.zeros_like(_workspace(xs))
        # our tile configurations: the default 128x128 and the 256x128 ones (fewer, larger tiles:
        # less wave quantization on e.g. 14x14x256, 1.5 rounds of 128x128 tiles)
        best = None
        for eng in (FWD_ENGINES if G.ENGINE == 0 else (0,)):
            t = _time_us(lambda: conv3x3_fwd(xs, w, stats=ws, engine=eng))
            if best is None or t < best[0]:
                best = (t, eng)
        theirs = _time_us(lambda: torch.nn.functional.conv2d(xs, w, None, 1, 1))
    n, _, h, wd = x.shape
    stats_pass_us = n * h * wd * weight.shape[0] * x.element_size() / 5e12 * 1e6
    choice = best[0] <= theirs + stats_pass_us
    _FWD_CHOICE[key] = choice
    _FWD_ENGINE[key] = best[1]
    return choice


def conv3x3(x, weight, with_stats=False, bnlink=None, gradlink=None):
    """Returns the conv output. If the forward runs on our kernel (:func:`conv3x3_forward_is_ours`)
    and ``with_stats``, its per-channel sum / sumsq are pending in the BatchNorm workspace
    (consume them with ``bn_from_stats(..., stats_ready=True)``); check with
    ``conv3x3_forward_is_ours`` first. ``gradlink`` (:class:`GradLink`): x's other consumer
    deposits its gradient of x there; the input gradient adds it in the dgrad epilogue."""
    ours = conv3x3_forward_is_ours(x, weight)
    return _Conv3x3.apply(x, weight, ours, with_stats and ours, bnlink, gradlink)


def conv3x3_fwd_raw(x, weight):
    """The 3x3 / s1 forward the autograd path would run (per-shape choice), without autograd."""
    x = x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)
    # a forward marks the cached transposed filter stale whichever kernel runs (as _Conv3x3 does):
    # the next input gradient re-derives it from the current weights
    note_filter(weight)
    if conv3x3_forward_is_ours(x, weight):
        return conv3x3_fwd(x, weight, engine=_FWD_ENGINE.get((tuple(x.shape), weight.shape[0])))
    return torch.nn.functional.conv2d(x, weight, None, 1, 1)


def conv3x3_dgrad_raw(dy, weight, x_shape, residual=None):
    """The 3x3 / s1 input gradient (+ ``residual`` in the epilogue) per the per-shape choice,
    without autograd."""
    if not dy.is_contiguous(memory_format=torch.channels_last):
        dy = dy.contiguous(memory_format=torch.channels_last)
    if _dgrad_is_ours(dy, weight, x_shape):
        return conv3x3_dgrad(dy, weight, residual=residual)
    xe = torch.empty(x_shape, device=dy.device, dtype=dy.dtype).contiguous(memory_format=torch.channels_last)
    dx = torch.ops.aten.convolution_backward(dy, xe, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                             [True, False, False])[0]
    return dx + residual if residual is not None else dx


def masked_links_ok() -> bool:
    """GradLinks may carry (dy, mask) instead of dres: the LDS-DMA dgrad kernel masks in its epilogue."""
    return G.ENGINE != 1


def conv1x1_stats(x, weight, link=None, bnlink=None):
    return _Conv1x1Stats.apply(x, weight, link, bnlink)


def conv1x1_forward_is_ours(x, weight) -> bool:
    """Per-shape choice of a 1x1 forward, measured once: our GEMM with the statistics epilogue
    vs MIOpen plus the statistics pass the next BatchNorm then needs (one read of the output
    at 5 TB/s)."""
    if CONV1X1 != "ours":
        return False
    def make():
        xs, w = x.detach().contiguous(memory_format=torch.channels_last), weight.detach()
        n, _, h, wd = xs.shape
        ws = torch.zeros_like(_workspace(xs))
        return (lambda: _fwd1x1_stats(xs, w, ws), lambda: torch.nn.functional.conv2d(xs, w),
                n * h * wd * w.shape[0] * xs.element_size())
    return stats_choice(_FWD1_CHOICE, (tuple(x.shape), weight.shape[0]), make)


def conv1x1_hybrid(x, weight, link=None, bnlink=None, ours_stats=False):
    """``ours_stats``: forward on our GEMM with the next BatchNorm's statistics left pending in
    the workspace (``bn_from_stats(..., stats_ready=True)``); else MIOpen's forward."""
    return _Conv1x1Hybrid.apply(x, weight, link, bnlink, ours_stats)


def bn_from_stats(x, bn, relu=False, residual=None, stats_ready=True, link=None, bnlink=None):
    mom, nbt = bn_counter(bn)
    return _BNFromStats.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var, mom, bn.eps, relu,
                              stats_ready, link, nbt, bnlink)


def bn_relu_conv1x1(c2, bn, weight, stats_ready=False):
    """conv1x1(relu(bn(c2)), W) with the BatchNorm + ReLU applied in the GEMM's A load (``stats_ready``:
    c2's sums are pending in the workspace from the GEMM that produced it)."""
    mom, nbt = bn_counter(bn)
    return _BNReluConv1x1.apply(c2, bn.weight, bn.bias, bn.running_mean, bn.running_var, weight, mom, bn.eps, nbt,
                                stats_ready)


def supported(x: torch.Tensor, *channels: int) -> bool:
    """Shapes the fused path handles (bf16 NHWC on GPU, channels % 32 == 0, <= 2048)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and all(c % 32 == 0 and 32 <= c <= 2048 for c in channels))
