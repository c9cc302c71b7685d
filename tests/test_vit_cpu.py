"""ViT pieces that run on the CPU: the one-pass [CLS] + position embedding and a tiny model's
forward / backward through the PyTorch paths."""
import torch

from fluxmpi_amd.models.vit import cls_pos, vit_tiny


def test_cls_pos_matches_concat_add():
    torch.manual_seed(0)
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(3, 5, 8).to(dt)
        cls, pos = torch.randn(1, 1, 8), torch.randn(1, 6, 8)
        ref = torch.cat([cls.expand(3, -1, -1).to(dt), x], 1) + pos.to(dt)
        assert torch.equal(cls_pos(x, cls, pos), ref)


def test_vit_tiny_forward_backward_cpu():
    torch.manual_seed(0)
    m = vit_tiny(num_classes=10, img=32)
    x = torch.randn(2, 3, 32, 32)
    y = m(x)
    assert y.shape == (2, 10) and torch.isfinite(y).all()
    y.sum().backward()
    assert m.cls.grad is not None and m.pos.grad is not None and torch.isfinite(m.pos.grad).all()
