"""MFMA stem (csrc/kernels/stem.hip) vs an fp32 PyTorch reference of
conv7x7/2 -> BatchNorm (training) -> ReLU -> max-pool 3x3/2: output, running statistics and
the gradients of the filter and the BatchNorm affine."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from fluxmpi_amd.ops import _ext
from fluxmpi_amd.ops import stem as S

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def _our_conv(x, w):
    """The stem kernel's conv output (NCHW view of the NHWC result) for the same inputs."""
    from fluxmpi_amd.ops.batchnorm import _workspace
    from fluxmpi_amd.ops.pool import pad_c3_to_c4
    C = _ext.get(required=True)
    n = x.shape[0]
    x4 = pad_c3_to_c4(x).permute(0, 2, 3, 1)
    c = torch.empty(n, 112, 112, 64, device=x.device, dtype=torch.bfloat16)
    ws = torch.zeros_like(_workspace(x))  # a scratch accumulator: the shared one stays zeroed
    C.stem_fwd(x4.data_ptr(), S.pack_filter(w).data_ptr(), c.data_ptr(), ws.data_ptr(), n,
               torch.cuda.current_stream().cuda_stream)
    sums = ws[: 64 * 2 * 64].reshape(64, 2, 64).sum(0)  # shards with channel stride 64
    cf = c.float().reshape(-1, 64)
    assert _rel(sums[0], cf.sum(0)) < 1e-4 and _rel(sums[1], (cf * cf).sum(0)) < 1e-4
    return c.float().permute(0, 3, 1, 2)


@pytest.mark.parametrize("n", [2, 5])
def test_stem_matches_reference(n):
    assert _ext.get(required=True) is not None
    torch.manual_seed(n)
    dev = "cuda"
    x = torch.randn(n, 3, 224, 224, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    bn = nn.BatchNorm2d(64).to(dev)
    with torch.no_grad():
        conv.weight.mul_(2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.2)
    assert S.supported(x, conv.weight, conv, bn)
    w_ref = conv.weight.detach().clone().requires_grad_(True)
    g_ref = bn.weight.detach().clone().requires_grad_(True)
    b_ref = bn.bias.detach().clone().requires_grad_(True)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()

    c_ours = _our_conv(x, conv.weight.detach())
    y = S.stem(x, conv, bn)
    c = F.conv2d(x.float(), w_ref, stride=2, padding=3)
    assert _rel(c_ours, c) < 1e-2, _rel(c_ours, c)
    # The max-pool argmax and the ReLU gate are discontinuous: one-ulp differences of the bf16
    # conv output flip near-tie windows, and each flip moves a whole gradient element (the
    # filter gradient moves by several % at this batch). So the reference pools on the kernel's
    # own conv output (straight-through: the gradient still flows through conv2d into w_ref).
    c = c + (c_ours - c).detach()
    ref = F.max_pool2d(F.relu(F.batch_norm(c, rm, rv, g_ref, b_ref, True, 0.1, bn.eps)), 3, 2, 1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 2e-2, _rel(y, ref)
    assert _rel(bn.running_mean, rm) < 2e-2 and _rel(bn.running_var, rv) < 2e-2
    assert int(bn.num_batches_tracked) == 1

    gy = torch.randn_like(ref)
    (y.float() * gy).sum().backward()
    (ref * gy).sum().backward()
    torch.cuda.synchronize()
    for got, want, name in ((conv.weight.grad, w_ref.grad, "conv"), (bn.weight.grad, g_ref.grad, "gamma"),
                            (bn.bias.grad, b_ref.grad, "beta")):
        assert got is not None and got.shape == want.shape, name
        assert _rel(got, want) < 3e-2, (name, _rel(got, want))


def test_stem_bwd_deterministic():
    torch.manual_seed(3)
    x = torch.randn(3, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda()
    bn = nn.BatchNorm2d(64).cuda()
    outs = []
    for _ in range(2):
        conv.weight.grad = None
        y = S.stem(x, conv, bn)
        y.float().square().sum().backward()
        outs.append(conv.weight.grad.clone())
    assert torch.equal(outs[0], outs[1]) or _rel(outs[0], outs[1]) < 1e-5

