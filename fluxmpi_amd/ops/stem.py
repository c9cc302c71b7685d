"""ResNet stem (7x7/2 conv -> BatchNorm -> ReLU -> 3x3/2 max-pool) on the MFMA stem kernels.

``stem(x, conv_weight, bn)`` == ``max_pool2d(relu(bn(conv2d(x, w, stride=2, padding=3))), 3, 2, 1)``
for 224x224 bf16 NHWC images in training mode (``csrc/kernels/stem.hip``):

* forward: the input channels are zero-padded 3 -> 4 (one pass), the convolution runs as an
  implicit GEMM over LDS image halos (no im2col) with the BatchNorm statistics reduced in its
  epilogue, then the fused BN + ReLU + max-pool of :mod:`.pool`;
* backward: ONE pass computes the pool-gradient gather, the BatchNorm backward sums and the
  three GEMMs the filter gradient decomposes into (``dW' = a*dz^T A + b*x^T A + d*colsum(A)``),
  then a small combine kernel; the gradient of the conv output is never materialised.

The convolution uses a packed filter ``W'[64][256]`` (K = 32 chunks of (ay, by, ax) x 8 elements
of (bx, c), see the kernel header); :func:`pack_maps` builds the gather index for the filter and
the inverse map that folds ``dW'`` back to ``[64, Cin, 7, 7]``. :func:`emulate_conv` evaluates
the same K layout with plain torch ops (CPU test of the layout, any image size).

Parity: the reference's model zoo trains Lux/Flux ResNets through FluxMPI's DDP wrapper
(``/root/reference/README.md``); this module is an MI355X-specific fusion of their stem.
"""
from __future__ import annotations

import functools

import torch

from . import _ext
from . import graddst
from .batchnorm import _workspace
from .multi_tensor import DTYPE_CODE

CO, KK = 64, 256


def _row_channel(r: int) -> int:
    """Output channel held by packed filter row r (a lane's 16 accumulators = 16 consecutive channels)."""
    return 16 * ((r >> 2) & 3) + 4 * (r >> 4) + (r & 3)


def _k_tap(k: int):
    """K index -> (ci, ky, kx) of the 7x7 filter, or None for a zero (padding) entry."""
    kc, e = k >> 3, k & 7
    ay, ax, by = kc & 3, (kc >> 2) & 3, kc >> 4
    bx, ci = e >> 2, e & 3
    ky, kx = 2 * ay + by - 1, 2 * ax + bx - 1
    if not (0 <= ky <= 6 and 0 <= kx <= 6):
        return None
    return ci, ky, kx


@functools.lru_cache(maxsize=8)
def _maps_cpu(cin: int):
    fwd = torch.full((CO, KK), -1, dtype=torch.long)
    bwd = torch.empty(CO, cin, 7, 7, dtype=torch.long)
    for k in range(KK):
        t = _k_tap(k)
        if t is None or t[0] >= cin:
            continue
        ci, ky, kx = t
        for r in range(CO):
            co = _row_channel(r)
            fwd[r, k] = ((co * cin + ci) * 7 + ky) * 7 + kx
        bwd[:, ci, ky, kx] = torch.arange(CO) * KK + k
    zero = CO * cin * 49  # index of an appended zero
    fwd = torch.where(fwd < 0, torch.full_like(fwd, zero), fwd)
    return fwd, bwd


_MAPS: dict = {}


def pack_maps(cin: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    """(fwd [64, 256]: flat filter index per packed entry, the appended zero for padding;
    bwd [64, cin, 7, 7]: flat index into dW' [64, 256] with natural channel rows)."""
    key = (cin, str(device))
    if key not in _MAPS:
        f, b = _maps_cpu(cin)
        _MAPS[key] = (f.to(device), b.to(device))
    return _MAPS[key]


def pack_filter(w: torch.Tensor) -> torch.Tensor:
    """[64, cin, 7, 7] -> packed W' [64, 256] (rows in the kernel's channel order), bf16."""
    fwd, _ = pack_maps(w.shape[1], w.device)
    flat = torch.cat([w.reshape(-1).to(torch.bfloat16), w.new_zeros(1, dtype=torch.bfloat16)])
    return flat[fwd].contiguous()


def unpack_grad(dwp: torch.Tensor, cin: int) -> torch.Tensor:
    """dW' [64, 256] (natural channel rows) -> dW [64, cin, 7, 7]."""
    _, bwd = pack_maps(cin, dwp.device)
    return dwp.reshape(-1)[bwd]


def emulate_conv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The stem convolution evaluated through the packed K layout with torch ops (fp32, NCHW in/out):
    A[p][k] gathered from the 4-channel padded image as the kernel's chunks do, times W'^T,
    rows put back in channel order. For tests of the layout; any even image size."""
    n, cin, h, wd = x.shape
    x4 = torch.zeros(n, h, wd, 4, dtype=torch.float32)
    x4[..., :cin] = x.float().permute(0, 2, 3, 1)
    oh, ow = h // 2, wd // 2
    cols = []
    for k in range(KK):
        kc, e = k >> 3, k & 7
        ay, ax, by = kc & 3, (kc >> 2) & 3, kc >> 4
        bx, c = e >> 2, e & 3
        iy = 2 * torch.arange(oh) + 2 * ay + by - 4
        ix = 2 * (torch.arange(ow) + ax) - 4 + bx
        vy = (iy >= 0) & (iy < h)
        vx = (ix >= 0) & (ix < wd)
        g = x4[:, iy.clamp(0, h - 1)][:, :, ix.clamp(0, wd - 1), c]
        g = g * (vy[:, None] & vx[None, :]).float()
        cols.append(g.reshape(n, oh * ow))
    a = torch.stack(cols, -1)  # [n, pixels, 256]
    flat = torch.cat([w.reshape(-1).float(), torch.zeros(1)])
    wp = flat[_maps_cpu(cin)[0]]  # [64 rows, 256]
    y_rows = a @ wp.t()  # [n, pixels, rows]
    perm = torch.tensor([_row_channel(r) for r in range(CO)])
    y = torch.empty_like(y_rows)
    y[..., perm] = y_rows
    return y.reshape(n, oh, ow, CO).permute(0, 3, 1, 2)


def supported(x: torch.Tensor, weight: torch.Tensor, conv, bn) -> bool:
    return (x.is_cuda and not x.requires_grad and x.dtype == torch.bfloat16 and x.dim() == 4
            and tuple(x.shape[1:]) == (3, 224, 224) and x.permute(0, 2, 3, 1).is_contiguous()
            and x.data_ptr() % 16 == 0 and tuple(weight.shape) == (CO, 3, 7, 7)
            and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3) and conv.bias is None
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1 and bn.training
            and bn.num_features == CO and _ext.available())


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x4, weight, bn_w, bn_b, running_mean, running_var, momentum, eps, nbt=None):
        C = _ext.get(required=True)
        n = x4.shape[0]
        stream = torch.cuda.current_stream(x4.device).cuda_stream
        wp = pack_filter(weight)
        c = torch.empty(n, 112, 112, CO, device=x4.device, dtype=torch.bfloat16)
        ws = _workspace(x4)
        C.stem_fwd(x4.data_ptr(), wp.data_ptr(), c.data_ptr(), ws.data_ptr(), n, stream)
        w32 = bn_w.float() if bn_w is not None else torch.ones(CO, device=x4.device)
        b32 = bn_b.float() if bn_b is not None else torch.zeros(CO, device=x4.device)
        mean = torch.empty(CO, device=x4.device, dtype=torch.float32)
        inv, scale, shift = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
        rm = running_mean.data_ptr() if running_mean is not None else 0
        rv = running_var.data_ptr() if running_var is not None else 0
        C.bn_stats_finalize(c.data_ptr(), w32.data_ptr(), b32.data_ptr(), rm, rv, mean.data_ptr(), inv.data_ptr(),
                            scale.data_ptr(), shift.data_ptr(), ws.data_ptr(), n * 112 * 112, CO, float(momentum),
                            float(eps), 1, DTYPE_CODE[torch.bfloat16], stream,
                            nbt.data_ptr() if nbt is not None else 0)
        y = torch.empty(n, 56, 56, CO, device=x4.device, dtype=torch.bfloat16)
        idx = torch.empty(n * 56 * 56 * CO, device=x4.device, dtype=torch.uint8)
        C.bn_relu_maxpool_fwd(c.data_ptr(), scale.data_ptr(), shift.data_ptr(), y.data_ptr(), idx.data_ptr(), n, 112,
                              112, CO, 3, 2, 1, DTYPE_CODE[torch.bfloat16], stream)
        ctx.save_for_backward(x4, c, idx, w32, mean, inv)
        ctx.dtypes = (weight.dtype, bn_w.dtype if bn_w is not None else None, bn_b is not None)
        ctx.params = (weight, bn_w, bn_b)  # the leaves: their gradients' DDP bucket slices (graddst)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.get(required=True)
        x4, c, idx, w32, mean, inv = ctx.saved_tensors
        n = x4.shape[0]
        dev = x4.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        dy = dy.permute(0, 2, 3, 1)
        if not dy.is_contiguous():
            dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        blocks = C.stem_bwd_blocks(n)
        part = torch.empty(blocks * C.stem_part_floats(), device=dev, dtype=torch.float32)
        weight, bn_w, bn_b = ctx.params
        need = ctx.needs_input_grad

        def bn_out(p, i):  # fp32 BN parameter gradients straight into their bucket slices
            t = graddst.take(p, (CO,), torch.float32) if need[i] else None
            return t if t is not None else torch.empty(CO, device=dev, dtype=torch.float32)

        dw_bn, db_bn = bn_out(bn_w, 2), bn_out(bn_b, 3)
        dwp = torch.empty(CO, KK, device=dev, dtype=torch.float32)
        C.stem_bwd(x4.data_ptr(), c.data_ptr(), dy.data_ptr(), idx.data_ptr(), w32.data_ptr(), mean.data_ptr(),
                   inv.data_ptr(), part.data_ptr(), blocks, _workspace(x4).data_ptr(), dw_bn.data_ptr(),
                   db_bn.data_ptr(), dwp.data_ptr(), n, stream)
        wdt, bdt, has_b = ctx.dtypes
        dw = None
        if need[1]:  # the unpack's cast writes the filter's bucket slice (in the filter's strides)
            dw = graddst.empty_like(weight, wdt)
            dw.copy_(unpack_grad(dwp, 3))
        return (None, dw, dw_bn.to(bdt) if bdt is not None else None, db_bn.to(bdt) if has_b else None,
                None, None, None, None, None)


def stem(x: torch.Tensor, conv, bn) -> torch.Tensor:
    """``max_pool2d(relu(bn(conv(x))), 3, 2, 1)`` on the stem kernels (see :func:`supported`)."""
    from .batchnorm import bn_counter
    from .pool import pad_c3_to_c4
    mom, nbt = bn_counter(bn)
    x4 = pad_c3_to_c4(x).permute(0, 2, 3, 1)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return _StemFn.apply(x4, conv.weight, bn.weight, bn.bias, rm, rv, mom, bn.eps, nbt)


__all__ = ["stem", "supported", "pack_filter", "unpack_grad", "pack_maps", "emulate_conv"]
