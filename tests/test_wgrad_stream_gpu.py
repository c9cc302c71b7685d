"""Weight gradients on the side stream (fluxmpi_amd/ops/streams.py, opt-in): ResNet / ViT
training steps give the same gradients with the side stream on and off, and the gradients are
complete when backward returns (the end-of-backward join)."""
import pytest
import torch

from fluxmpi_amd.ops import streams

pytestmark = pytest.mark.gpu


def _grads(model, x, y, on):
    saved = streams.ENABLED
    streams.ENABLED = on
    try:
        for p in model.parameters():
            p.grad = None
        loss = torch.nn.functional.cross_entropy(model(x).float(), y)
        loss.backward()
        # read the gradients right away on the current stream: must see finished values
        out = [p.grad.float().clone() for p in model.parameters() if p.grad is not None]
        assert all(torch.isfinite(g).all() for g in out)
        return out
    finally:
        streams.ENABLED = saved


@pytest.mark.parametrize("name", ["resnet", "vit"])
def test_side_stream_grads_match(name):
    torch.manual_seed(0)
    torch.backends.cudnn.deterministic = True
    if name == "resnet":
        from fluxmpi_amd.models import resnet
        model = resnet.resnet18ish(num_classes=10, conv_impl="hybrid", norm="fused").cuda().to(
            memory_format=torch.channels_last)
        for m in model.modules():  # bf16 weights, fp32 BatchNorm (as bench.py / smoke())
            if not isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                for p in m.parameters(recurse=False):
                    p.data = p.data.to(torch.bfloat16)
        x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), device="cuda")
    else:
        from fluxmpi_amd.models import vit
        model = vit.ViT(img=32, patch=8, dim=128, depth=2, heads=4, mlp=256, num_classes=10).cuda().bfloat16()
        x = torch.randn(64, 3, 32, 32, device="cuda").bfloat16()  # 64 x 17 tokens: the HIP wgrad path
        y = torch.randint(0, 10, (64,), device="cuda")
    g_on = _grads(model, x, y, True)
    g_off = _grads(model, x, y, False)
    assert len(g_on) == len(g_off) > 0
    for a, b in zip(g_on, g_off):
        assert torch.allclose(a, b, rtol=2e-2, atol=2e-2 * float(b.abs().max()) + 1e-6)
