"""ResNet-50 (He et al. 2016; torchvision layout) for the north-star benchmark.

The reference's headline workload is the Lux.jl ImageNet ResNet-50 example
(``README.md:74-78``, ``BASELINE.json`` "ResNet50 Lux.jl DDP"). There is no
torchvision in this image, so the architecture is written out here:
7x7/2 stem -> 3x3/2 max-pool -> bottleneck stages [3, 4, 6, 3] (width 64..512,
expansion 4, stride on the 3x3 conv, "ResNet v1.5") -> global average pool ->
1000-way FC. 25.56 M parameters, 161 parameter tensors.

MI355X choices:

* activations in ``channels_last`` (NHWC): channels innermost is what the
  conv kernels and our NHWC BatchNorm kernels want, and it makes every 1x1
  convolution a plain GEMM ``[N*H*W, Cin] x [Cin, Cout]``;
* ``conv_impl="gemm"`` routes 1x1 convolutions (36 of the 53 convs) to
  hipBLASLt matmuls on that NHWC view instead of MIOpen;
* ``norm="fused"`` uses the hand-written gfx950 NHWC BatchNorm kernels with
  the ReLU (and the residual add of each block) fused into the normalisation
  pass (``fluxmpi_amd.ops.batchnorm``); ``norm="torch"`` uses ``nn.BatchNorm2d``.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.linear import Linear

# ResNet stem: "ours" = the MFMA stem kernels (ops/stem.py: conv + BN statistics forward, one fused
# backward pass) when the input is a 224x224 bf16 NHWC batch; "miopen" = padded MIOpen conv + the
# fused BN/ReLU/max-pool of ops/pool.py
STEM = os.environ.get("FLUXMPI_STEM", "ours")


class Conv1x1(nn.Module):
    """1x1 convolution computed as a GEMM on the NHWC view (hipBLASLt)."""

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.stride = stride
        self.weight = nn.Parameter(torch.empty(cout, cin, 1, 1))
        nn.init.kaiming_normal_(self.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        if self.stride != 1:
            x = x[:, :, ::self.stride, ::self.stride]
        n, c, h, w = x.shape
        # NHWC memory -> [N*H*W, C] without a copy when x is channels_last
        xm = x.permute(0, 2, 3, 1).reshape(n * h * w, c)
        y = torch.matmul(xm, self.weight.view(self.weight.shape[0], c).t())
        return y.view(n, h, w, -1).permute(0, 3, 1, 2)


class _GlobalAvgPool(torch.autograd.Function):
    """``x.mean((2, 3))`` whose backward writes the broadcast ``dy / (H*W)`` straight into a
    gradient with x's memory format (one write pass). ``adaptive_avg_pool2d``'s backward on
    a channels_last input is an NCHW expand + divide + layout copy: ~100 us per ResNet-50
    step on MI355X (s47 trace) for a 51 MB gradient."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        ctx.cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.shape
        g = (dy / (h * w)).to(dy.dtype)
        if ctx.cl:
            out = torch.empty((n, h, w, c), device=dy.device, dtype=dy.dtype)
            out.copy_(g[:, None, None, :].expand(n, h, w, c))
            return out.permute(0, 3, 1, 2)
        return g[:, :, None, None].expand(n, c, h, w).contiguous()


def global_avg_pool(x):
    """``flatten(adaptive_avg_pool2d(x, 1), 1)`` with a single-pass backward."""
    return _GlobalAvgPool.apply(x)


def conv1x1(cin, cout, stride=1, impl="gemm"):
    if impl == "gemm":
        return Conv1x1(cin, cout, stride)
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _norm(c, kind):
    if kind == "fused":
        from ..ops.batchnorm import FusedBatchNorm2d
        return FusedBatchNorm2d(c)
    return nn.BatchNorm2d(c)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None, conv_impl="gemm", norm="torch"):
        super().__init__()
        cout = width * self.expansion
        # "fused": 1x1 convs run on our MFMA GEMM with BatchNorm producer/consumer fusion
        # (fluxmpi_amd.ops.fused_block); parameters are plain Conv2d/BatchNorm modules.
        # "hybrid": MIOpen forward/wgrad for the 1x1 convs, our dgrad GEMM with the block's
        # residual gradient added in its epilogue (fluxmpi_amd.ops.fused_block.conv1x1_hybrid)
        self.gemm_fused = conv_impl == "fused"
        self.hybrid = conv_impl == "hybrid"
        if self.gemm_fused or self.hybrid:
            conv_impl, norm = "miopen", "fused"
        self.dims = (cin, width, cout)
        self.conv1 = conv1x1(cin, width, 1, conv_impl)
        self.bn1 = _norm(width, norm)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = _norm(width, norm)
        self.conv3 = conv1x1(width, cout, 1, conv_impl)
        self.bn3 = _norm(cout, norm)
        self.downsample = downsample
        self.fused = norm == "fused"

    def _fused_downsample(self) -> bool:
        ds = self.downsample
        return (ds is not None and len(ds) == 2 and isinstance(ds[0], nn.Conv2d) and ds[0].kernel_size == (1, 1)
                and ds[0].bias is None and ds[0].padding == (0, 0) and ds[0].stride[0] == ds[0].stride[1]
                and ds[0].groups == 1 and ds[0].dilation == (1, 1))

    def forward(self, x):
        if (self.gemm_fused or self.hybrid) and self.training:
            from ..ops import fused_block as fb
            if fb.supported(x, *self.dims):
                grad = torch.is_grad_enabled()
                needs = x.requires_grad and grad
                # identity blocks: bn3's residual gradient goes straight into conv1's dgrad epilogue,
                # and that epilogue (whose output is then the whole gradient of the previous
                # block's output) also reduces the previous block's bn3 backward statistics.
                # downsample blocks: the downsample conv's input gradient goes into that epilogue.
                fused_ds = self.downsample is not None and self._fused_downsample()
                if self.downsample is None:
                    # masked: bn3 hands over (dy, relu mask); conv1's dgrad epilogue applies the mask
                    link = fb.GradLink(masked=fb.masked_links_ok()) if needs else None
                else:
                    link = fb.SideGradLink() if (needs and fused_ds) else None
                # (BatchNorm-backward reductions in the dgrad epilogues — fused_block.BNStatsLink —
                # measured a loss in every form on MI355X, round 4: not linked here)
                if self.hybrid:
                    o1 = fb.conv1x1_forward_is_ours(x, self.conv1.weight)
                    c1 = fb.conv1x1_hybrid(x, self.conv1.weight, link, ours_stats=o1)
                    a1 = fb.bn_from_stats(c1, self.bn1, relu=True, stats_ready=True) if o1 else \
                        self.bn1(c1, relu=True)
                else:
                    c1 = fb.conv1x1_stats(x, self.conv1.weight, link)  # + bn1 statistics (GEMM epilogue)
                    a1 = fb.bn_from_stats(c1, self.bn1, relu=True)
                # the downsample branch is built AFTER conv1: autograd runs ready nodes newest-first
                # and conv1's backward becomes ready last, so the downsample conv's backward (which
                # offers its input gradient to conv1's dgrad through the SideGradLink) runs before
                # it. (And after bn1 consumed conv1's epilogue statistics: the downsample BN uses
                # the same statistics workspace.)
                cds = None  # downsample conv output whose BN is fused into bn3 (dual_bn_relu)
                if self.downsample is None:
                    identity = x
                elif fused_ds:
                    ds = self.downsample
                    dual = fb.dual_bn_ok(x, ds[0].out_channels, self.bn3, ds[1])
                    # our GEMM (+ the downsample BN's sums in its epilogue) where measured faster
                    ds_stats = dual and fb.ds_forward_is_ours(x, ds[0].weight, ds[0].stride[0])
                    identity = fb.conv1x1_downsample(x, ds[0].weight, ds[0].stride[0],
                                                     link if isinstance(link, fb.SideGradLink) else None,
                                                     ours_stats=ds_stats)
                    if dual:
                        cds, identity = identity, None
                    else:
                        identity = ds[1](identity)
                else:
                    identity = self.downsample(x)
                if self.hybrid:
                    if fb.conv3x3_supported(a1, self.conv2):
                        # implicit-GEMM conv2 (input gradient always; forward where measured faster,
                        # then bn2's statistics come from its epilogue)
                        ours = fb.conv3x3_forward_is_ours(a1, self.conv2.weight)
                        c2 = fb.conv3x3(a1, self.conv2.weight, with_stats=True)
                        a2 = fb.bn_from_stats(c2, self.bn2, relu=True, stats_ready=ours)
                    elif fb.conv3x3_s2_supported(a1, self.conv2):
                        # stride-2 conv2: forward where measured faster on our implicit GEMM (+ bn2's
                        # sums from its epilogue), weight gradient autotuned (fused_block._Conv3x3S2)
                        ours = fb.conv3x3_s2_forward_is_ours(a1, self.conv2.weight)
                        c2 = fb.conv3x3_s2(a1, self.conv2.weight, with_stats=ours)
                        a2 = fb.bn_from_stats(c2, self.bn2, relu=True, stats_ready=ours)
                    else:
                        a2 = self.bn2(self.conv2(a1), relu=True)
                    o3 = fb.conv1x1_forward_is_ours(a2, self.conv3.weight)
                    c3 = fb.conv1x1_hybrid(a2, self.conv3.weight, None, ours_stats=o3)
                else:
                    c2 = fb.conv3x3(a1, self.conv2.weight) if fb.conv3x3_supported(a1, self.conv2) else self.conv2(a1)
                    c3 = fb.bn_relu_conv1x1(c2, self.bn2, self.conv3.weight)  # bn2+relu fused into the A load
                if cds is not None:
                    out = fb.dual_bn_relu(c3, self.bn3, cds, self.downsample[1],
                                          stats_ready=o3 if self.hybrid else True, ds_stats_ready=ds_stats)
                elif self.hybrid and not o3:
                    out = self.bn3(c3, relu=True, residual=identity, link=link if self.downsample is None else None)
                elif self.hybrid:
                    out = fb.bn_from_stats(c3, self.bn3, relu=True, residual=identity, stats_ready=True,
                                           link=link if self.downsample is None else None)
                else:
                    out = fb.bn_from_stats(c3, self.bn3, relu=True, residual=identity,
                                           link=link if self.downsample is None else None)
                return out
        identity = x if self.downsample is None else self.downsample(x)
        if self.fused:
            out = self.bn1(self.conv1(x), relu=True)
            out = self.bn2(self.conv2(out), relu=True)
            return self.bn3(self.conv3(out), relu=True, residual=identity)
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return F.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, conv_impl="gemm", norm="torch", zero_init_residual=False):
        super().__init__()
        if conv_impl in ("fused", "hybrid"):
            norm = "fused"
        self.conv_impl, self.norm_kind = conv_impl, norm
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _norm(64, norm)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(64, layers[0], 1)
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        # ops.linear.Linear: its backward writes dW / db into their DDP bucket slices (graddst)
        self.fc = Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _stem_conv(self, x):
        """7x7/2 stem. On the GPU the 3 input channels are zero-padded to 4 (image and
        filter; same math, and the filter's gradient is the slice of the padded one):
        MIOpen's NHWC kernels for C=4 run the forward 1.3x and the weight gradient 1.4x
        faster than for C=3 on MI355X (scripts/bench_stem.py), for one ~30 us pad pass."""
        w = self.conv1.weight
        if not (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and w.shape[1] == 3
                and self.conv_impl in ("hybrid", "fused")):
            return self.conv1(x)
        w4 = F.pad(w, (0, 0, 0, 0, 0, 1)).contiguous(memory_format=torch.channels_last)
        if (not x.requires_grad and x.dtype in (torch.bfloat16, torch.float16)
                and x.permute(0, 2, 3, 1).is_contiguous() and x.data_ptr() % 16 == 0):
            from ..ops.pool import pad_c3_to_c4
            x4 = pad_c3_to_c4(x)  # one HIP pass (6 B read, 8 B written per pixel)
        else:
            n, _, h, wd = x.shape
            x4 = torch.empty(n, h, wd, 4, device=x.device, dtype=x.dtype)
            x4[..., 3] = 0
            x4[..., :3] = x.permute(0, 2, 3, 1)
            x4 = x4.permute(0, 3, 1, 2)
        return F.conv2d(x4, w4, None, self.conv1.stride, self.conv1.padding)

    def _make(self, width, blocks, stride):
        down = None
        cout = width * Bottleneck.expansion
        if stride != 1 or self.inplanes != cout:
            impl = "miopen" if self.conv_impl in ("fused", "hybrid") else self.conv_impl
            down = nn.Sequential(conv1x1(self.inplanes, cout, stride, impl), _norm(cout, self.norm_kind))
        mods = [Bottleneck(self.inplanes, width, stride, down, self.conv_impl, self.norm_kind)]
        self.inplanes = cout
        for _ in range(1, blocks):
            mods.append(Bottleneck(cout, width, 1, None, self.conv_impl, self.norm_kind))
        return nn.Sequential(*mods)

    def forward(self, x):
        if self.norm_kind == "fused":
            from ..ops import pool
            from ..ops import stem as stem_ops
            if (self.training and self.conv_impl in ("hybrid", "fused") and STEM == "ours"
                    and stem_ops.supported(x, self.conv1.weight, self.conv1, self.bn1)):
                # conv + BN statistics + BN/ReLU/max-pool on the MFMA stem kernels; the backward
                # is one fused pass (ops/stem.py)
                x = stem_ops.stem(x, self.conv1, self.bn1)
                x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
                return self.fc(global_avg_pool(x))
            c = self._stem_conv(x)
            if self.training and pool.supported(c):
                # BN + ReLU + 3x3/2 max-pool in one pass over the stem output
                x = pool.bn_relu_maxpool(c, self.bn1, 3, 2, 1)
            else:
                x = self.maxpool(self.bn1(c, relu=True))
        else:
            x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(global_avg_pool(x))


def resnet50(num_classes=1000, **kw) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes, **kw)


def resnet18ish(num_classes=10, **kw) -> ResNet:
    """Small bottleneck ResNet ([1,1,1,1]) for fast tests."""
    return ResNet((1, 1, 1, 1), num_classes, **kw)
