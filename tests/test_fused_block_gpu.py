"""GEMM+BatchNorm producer/consumer fusion vs the unfused bottleneck (GPU only, bf16)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _models(impl="fused"):
    from fluxmpi_amd.models.resnet import ResNet
    torch.manual_seed(0)
    ref = ResNet((2, 1, 1, 1), 10, conv_impl="miopen", norm="fused").cuda().to(memory_format=torch.channels_last)
    fus = ResNet((2, 1, 1, 1), 10, conv_impl=impl).cuda().to(memory_format=torch.channels_last)
    fus.load_state_dict(ref.state_dict())
    for m in (ref, fus):
        for mod in m.modules():
            if not isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
                for p in mod.parameters(recurse=False):
                    p.data = p.data.bfloat16()
    return ref, fus


@pytest.mark.parametrize("impl", ["fused", "hybrid"])
def test_fused_resnet_matches_unfused(gpu_ext, impl):
    """Both bf16 pipelines are compared with an fp32 model holding the same (bf16-rounded)
    weights: the fused pipeline must be about as accurate as the unfused one. Layer 1 has an
    identity block, so the GradLink residual-gradient hand-off is exercised; "fused" applies bn2 +
    ReLU in conv3's A load (bn_relu_conv1x1)."""
    from fluxmpi_amd.models.resnet import ResNet
    ref, fus = _models(impl)
    f32 = ResNet((2, 1, 1, 1), 10, conv_impl="miopen", norm="fused").cuda().to(memory_format=torch.channels_last)
    f32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ya, yb, yc = ref(x), fus(x), f32(x.float())
    assert _rel(yb, yc) < 2 * _rel(ya, yc) + 1e-2
    g = torch.randn_like(yc)
    for y, m in ((ya, ref), (yb, fus), (yc, f32)):
        (y.float() * g).sum().backward()
    for (n, pa), pb, pc in zip(ref.named_parameters(), fus.parameters(), f32.parameters()):
        ea, eb = _rel(pa.grad, pc.grad), _rel(pb.grad, pc.grad)
        assert eb < 2 * ea + 2e-2, f"{n}: fused {eb:.3e} vs unfused {ea:.3e}"
    for (n, b), c in zip(ref.named_buffers(), fus.buffers()):
        if b.dtype.is_floating_point:
            assert _rel(c, b) < 2e-2, n
        else:  # num_batches_tracked (incremented inside the finalize kernels)
            assert torch.equal(c, b) and int(b) == 1, n


def test_fused_ops_individually(gpu_ext):
    """conv1x1_stats + bn_from_stats == conv + FusedBatchNorm2d; bn_relu_conv1x1 likewise."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(1)
    x = torch.randn(4, 64, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 64, 1, 1, device="cuda") * 0.1).bfloat16()
    bn_a, bn_b = FusedBatchNorm2d(128).cuda(), FusedBatchNorm2d(128).cuda()
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    wa, wb = w.clone().requires_grad_(), w.clone().requires_grad_()
    ya = bn_a(torch.nn.functional.conv2d(xa, wa), relu=True)
    yb = fb.bn_from_stats(fb.conv1x1_stats(xb, wb), bn_b, relu=True)
    assert _rel(yb, ya) < 2e-2
    torch.testing.assert_close(bn_b.running_mean, bn_a.running_mean, rtol=1e-2, atol=1e-3)
    g = torch.randn_like(ya)
    (ya.float() * g).sum().backward()
    (yb.float() * g).sum().backward()
    assert _rel(xb.grad, xa.grad) < 3e-2 and _rel(wb.grad, wa.grad) < 3e-2
    # bn2 -> relu -> conv3 with the activation never materialised
    bn2a, bn2b = FusedBatchNorm2d(64).cuda(), FusedBatchNorm2d(64).cuda()
    w3 = (torch.randn(256, 64, 1, 1, device="cuda") * 0.1).bfloat16()
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    w3a, w3b = w3.clone().requires_grad_(), w3.clone().requires_grad_()
    za = torch.nn.functional.conv2d(bn2a(xa, relu=True), w3a)
    zb = fb.bn_relu_conv1x1(xb, bn2b, w3b)
    torch.cuda.synchronize()
    from fluxmpi_amd.ops.batchnorm import _workspace
    _workspace(xb).zero_()  # zb's statistics are pending in the workspace (no consumer here)
    assert _rel(zb, za) < 2e-2
    g = torch.randn_like(za)
    (za.float() * g).sum().backward()
    (zb.float() * g).sum().backward()
    assert _rel(xb.grad, xa.grad) < 3e-2 and _rel(w3b.grad, w3a.grad) < 3e-2
    assert _rel(bn2b.weight.grad, bn2a.weight.grad) < 3e-2


def test_hybrid_conv_with_link(gpu_ext):
    """relu(bn(conv1x1_hybrid(x)) + x) with the residual gradient handed over by a GradLink
    == the same block with autograd summing the two input gradients."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(2)
    x = torch.randn(4, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 1, 1, device="cuda") * 0.1).bfloat16()
    bn_a, bn_b = FusedBatchNorm2d(128).cuda(), FusedBatchNorm2d(128).cuda()
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    wa, wb = w.clone().requires_grad_(), w.clone().requires_grad_()
    ya = bn_a(torch.nn.functional.conv2d(xa, wa), relu=True, residual=xa)
    link = fb.GradLink()
    yb = bn_b(fb.conv1x1_hybrid(xb, wb, link), relu=True, residual=xb, link=link)
    assert _rel(yb, ya) < 1e-2  # batch statistics: float-atomic order differs between calls
    g = torch.randn_like(ya)
    (ya.float() * g).sum().backward()
    (yb.float() * g).sum().backward()
    assert link.grad is None  # consumed
    assert _rel(xb.grad, xa.grad) < 1e-2 and _rel(wb.grad, wa.grad) < 1e-2
    assert _rel(bn_b.weight.grad, bn_a.weight.grad) < 1e-4  # float atomics: order-dependent rounding


@pytest.mark.parametrize("impl", ["hybrid", "fused"])
def test_downsample_grad_delivered(gpu_ext, impl, monkeypatch):
    """Every downsample block (stride 1 in layer 1, stride 2 after) hands its input gradient to
    conv1's dgrad epilogue (autograd's newest-first order runs the downsample branch first), so
    no add kernel sums the block input's two gradients; the gradients equal the plain model's."""
    from fluxmpi_amd.ops import fused_block as fb
    links = []

    class Recording(fb.SideGradLink):
        __slots__ = ()

        def __init__(self):
            super().__init__()
            links.append(self)

    monkeypatch.setattr(fb, "SideGradLink", Recording)
    from fluxmpi_amd.models.resnet import ResNet
    ref, fus = _models(impl)
    f32 = ResNet((2, 1, 1, 1), 10, conv_impl="miopen", norm="fused").cuda().to(memory_format=torch.channels_last)
    f32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ya, yb, yc = ref(x), fus(x), f32(x.float())
    g = torch.randn_like(yc)
    for y in (ya, yb, yc):
        (y.float() * g).sum().backward()
    assert len(links) == 4 and all(lk.delivered and lk.grad is None for lk in links)
    for (n, pa), pb, pc in zip(ref.named_parameters(), fus.parameters(), f32.parameters()):
        ea, eb = _rel(pa.grad, pc.grad), _rel(pb.grad, pc.grad)
        assert eb < 2 * ea + 2e-2, f"{n}: linked {eb:.3e} vs unlinked {ea:.3e}"


@pytest.mark.parametrize("with_res", [False, True])
def test_bn_stats_link(gpu_ext, with_res):
    """BN -> 1x1 conv (its only consumer): the conv's dgrad epilogue reduces the BN backward
    statistics (ReLU mask recomputed, or the 1-bit mask after a residual add) and the BN
    skips its reduce pass — gradients equal the unlinked chain's."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(4)
    c = torch.randn(4, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(c) if with_res else None
    w = (torch.randn(64, 128, 1, 1, device="cuda") * 0.1).bfloat16()
    bn_w, bn_b = torch.rand(128, device="cuda") + 0.5, torch.rand(128, device="cuda") * 0.4 - 0.2
    grads = []
    for use_link in (False, True):
        bn = FusedBatchNorm2d(128).cuda()
        with torch.no_grad():
            bn.weight.copy_(bn_w)
            bn.bias.copy_(bn_b)
        ci, wi = c.clone().requires_grad_(), w.clone().requires_grad_()
        ri = r.clone().requires_grad_() if with_res else None
        link = fb.BNStatsLink() if use_link else None
        y = bn(ci, relu=True, residual=ri, bnlink=link)
        z = fb.conv1x1_hybrid(y, wi, None, link)
        (z.float() * torch.linspace(-1, 1, z.numel(), device="cuda").view_as(z)).sum().backward()
        if use_link:
            assert not link.bound  # consumed and released by the BN backward
        grads.append([ci.grad, wi.grad, bn.weight.grad, bn.bias.grad] + ([ri.grad] if with_res else []))
    for a, b in zip(*grads):
        assert _rel(b, a) < 2e-3, (_rel(b, a))


@pytest.mark.parametrize("wgrad", ["ours", "miopen"])
def test_hybrid_resnet_weight_gradient_kernels(gpu_ext, wgrad, monkeypatch):
    """The hybrid ResNet with every bottleneck weight gradient forced onto our split-K kernel
    (or MIOpen) matches the fp32 model as closely as the unfused bf16 pipeline does."""
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.ops import conv_choice as CC
    monkeypatch.setattr(CC, "WGRAD", wgrad)
    monkeypatch.setattr(CC, "_WG_CHOICE", {})
    ref, fus = _models("hybrid")
    f32 = ResNet((2, 1, 1, 1), 10, conv_impl="miopen", norm="fused").cuda().to(memory_format=torch.channels_last)
    f32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ya, yb, yc = ref(x), fus(x), f32(x.float())
    g = torch.randn_like(yc)
    for y in (ya, yb, yc):
        (y.float() * g).sum().backward()
    assert CC._WG_CHOICE and all(c[0] == wgrad for c in CC._WG_CHOICE.values())
    for (n, pa), pb, pc in zip(ref.named_parameters(), fus.parameters(), f32.parameters()):
        ea, eb = _rel(pa.grad, pc.grad), _rel(pb.grad, pc.grad)
        assert eb < 2 * ea + 2e-2, f"{n}: {wgrad} {eb:.3e} vs unfused {ea:.3e}"


@pytest.mark.parametrize("with_res", [False, True])
def test_bn_stats_link_conv3x3(gpu_ext, with_res):
    """BN -> 3x3 conv (implicit GEMM): the conv's dgrad epilogue reduces the BN backward
    statistics and the BN skips its reduce pass — gradients equal the unlinked chain's."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(7)
    c = torch.randn(4, 64, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(c) if with_res else None
    w = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    bn_w, bn_b = torch.rand(64, device="cuda") + 0.5, torch.rand(64, device="cuda") * 0.4 - 0.2
    grads = []
    for use_link in (False, True):
        bn = FusedBatchNorm2d(64).cuda()
        with torch.no_grad():
            bn.weight.copy_(bn_w)
            bn.bias.copy_(bn_b)
        ci, wi = c.clone().requires_grad_(), w.clone().requires_grad_()
        ri = r.clone().requires_grad_() if with_res else None
        link = fb.BNStatsLink() if use_link else None
        y = bn(ci, relu=True, residual=ri, bnlink=link)
        z = fb.conv3x3(y, wi, bnlink=link)
        if fb.conv3x3_forward_is_ours(y, wi):
            torch.cuda.synchronize()
        (z.float() * torch.linspace(-1, 1, z.numel(), device="cuda").view_as(z)).sum().backward()
        if use_link:
            assert not link.bound  # consumed and released by the BN backward
        grads.append([ci.grad, wi.grad, bn.weight.grad, bn.bias.grad] + ([ri.grad] if with_res else []))
    for a, b in zip(*grads):
        assert _rel(b, a) < 2e-3, (_rel(b, a))


def test_masked_grad_link(gpu_ext):
    """A masked GradLink hands (dy, relu mask) to conv1's dgrad epilogue, which applies the mask:
    the BatchNorm backward writes no dres, and the gradients equal the unmasked hand-off's."""
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(8)
    x = torch.randn(4, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 1, 1, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
    grads = []
    for masked in (False, True):
        bn = FusedBatchNorm2d(128).cuda()
        xi, wi = x.clone().requires_grad_(), w.clone().requires_grad_()
        link = fb.GradLink(masked=masked)
        y = bn(fb.conv1x1_hybrid(xi, wi, link), relu=True, residual=xi, link=link)
        (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        assert link.grad is None
        grads.append([xi.grad, wi.grad, bn.weight.grad, bn.bias.grad])
    for a, b in zip(*grads):  # the two forwards' batch statistics differ in float-atomic order only
        assert _rel(b, a) < 1e-3


@pytest.mark.parametrize("ch,hw", [(256, 14), (512, 7), (2048, 4)])
def test_dual_bn_relu(gpu_ext, ch, hw):
    """relu(bn3(c3) + bn_ds(c_ds)) through the dual kernels vs the fp32 composition: output,
    both inputs' gradients, both BatchNorms' parameter gradients and running statistics."""
    import torch.nn.functional as F
    from fluxmpi_amd.ops import fused_block as fb
    from fluxmpi_amd.ops.batchnorm import FusedBatchNorm2d
    torch.manual_seed(ch)
    cl = torch.channels_last
    c3 = (torch.randn(8, ch, hw, hw, device="cuda") * 2 + 0.5).bfloat16().contiguous(memory_format=cl)
    cds = (torch.randn(8, ch, hw, hw, device="cuda") * 0.7 - 0.3).bfloat16().contiguous(memory_format=cl)
    bn, bnd = FusedBatchNorm2d(ch).cuda(), FusedBatchNorm2d(ch).cuda()
    with torch.no_grad():
        for m in (bn, bnd):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
    rb = [t.clone() for t in (bn.running_mean, bn.running_var, bnd.running_mean, bnd.running_var)]
    a, b = c3.clone().requires_grad_(), cds.clone().requires_grad_()
    y = fb.dual_bn_relu(a, bn, b, bnd, stats_ready=False)
    g = torch.randn(y.shape, device="cuda")
    (y.float() * g).sum().backward()
    a32, b32 = c3.float().requires_grad_(), cds.float().requires_grad_()
    w1, b1, w2, b2 = (t.detach().clone().requires_grad_() for t in (bn.weight, bn.bias, bnd.weight, bnd.bias))
    rm1, rv1, rm2, rv2 = rb
    y32 = F.relu(F.batch_norm(a32, rm1, rv1, w1, b1, True, 0.1, 1e-5)
                 + F.batch_norm(b32, rm2, rv2, w2, b2, True, 0.1, 1e-5))
    (y32 * g).sum().backward()
    assert _rel(y, y32) < 1e-2
    for got, ref in ((a.grad, a32.grad), (b.grad, b32.grad), (bn.weight.grad, w1.grad), (bn.bias.grad, b1.grad),
                     (bnd.weight.grad, w2.grad), (bnd.bias.grad, b2.grad)):
        assert _rel(got, ref) < 2e-2
    for got, ref in ((bn.running_mean, rm1), (bn.running_var, rv1), (bnd.running_mean, rm2), (bnd.running_var, rv2)):
        assert _rel(got, ref) < 1e-3
    assert int(bn.num_batches_tracked) == 1 and int(bnd.num_batches_tracked) == 1


@pytest.mark.parametrize("impl", ["hybrid", "fused"])
@pytest.mark.parametrize("ds_fwd", ["miopen", "force"])
def test_resnet_dual_bn_matches_separate(gpu_ext, impl, ds_fwd, monkeypatch):
    """The ResNet downsample blocks with the dual BatchNorm vs the separate bn_ds + bn3 path,
    both measured against the fp32 model (bf16 gradients of a deep net differ by ~10-30% at
    the stem between any two bf16 pipelines; the dual one must be as accurate). ``force``: the
    downsample forward on our GEMM (stride-2 row gather) with bn_ds's sums from its epilogue."""
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.ops import fused_block as fb
    monkeypatch.setattr(fb, "DS_FWD", ds_fwd)
    outs = []
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    for dual in (False, True):
        monkeypatch.setattr(fb, "DUAL_BN", dual)
        ref, fus = _models(impl)
        y = fus(x)
        outs.append((y, fus))
    f32 = ResNet((2, 1, 1, 1), 10, conv_impl="miopen", norm="fused").cuda().to(memory_format=torch.channels_last)
    f32.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    yc = f32(x.float())
    g = torch.randn_like(yc)
    for y, m in outs + [(yc, f32)]:
        (y.float() * g).sum().backward()
    (ya, ma), (yb, mb) = outs
    assert _rel(yb, yc) < 2 * _rel(ya, yc) + 1e-2
    for (n, pa), pb, pc in zip(ma.named_parameters(), mb.parameters(), f32.parameters()):
        ea, eb = _rel(pa.grad, pc.grad), _rel(pb.grad, pc.grad)
        assert eb < 2 * ea + 2e-2, f"{n}: dual {eb:.3e} vs separate {ea:.3e}"
    for (n, a), b in zip(ma.named_buffers(), mb.buffers()):
        assert (torch.equal(a, b) if not a.dtype.is_floating_point else _rel(b, a) < 1e-2), n
