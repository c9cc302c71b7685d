"""DDP engine on the GPU (world of one over the native RCCL communicator): fused flat-bucket
optimiser vs the functional Optimisers path, HIP-graph replay vs eager."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mlp(seed, dev="cuda"):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64), torch.nn.Tanh(),
                               torch.nn.Linear(64, 1)).to(dev)


def test_ddp_gpu_matches_functional(gpu_ext):
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    m1, m2 = _mlp(0), _mlp(0)
    ddp = DDP(m1, O.Adam(1e-2), bucket_mb=0.004, first_bucket_mb=0.002)
    ps = {n: p.detach().clone() for n, p in m2.named_parameters()}
    st = O.setup(O.Adam(1e-2), ps)
    x = torch.randn(16, 32, device="cuda")
    y = x.sum(1, keepdim=True).sin()
    for _ in range(5):
        ((ddp(x) - y) ** 2).mean().backward()
        ddp.step()
        for n, p in m2.named_parameters():
            p.data.copy_(ps[n])
            p.grad = None
        ((m2(x) - y) ** 2).mean().backward()
        st, ps = O.update(st, ps, {n: p.grad for n, p in m2.named_parameters()})
    for n, p in m1.named_parameters():
        torch.testing.assert_close(p.detach(), ps[n], rtol=1e-5, atol=1e-6)


def test_graphed_step_matches_eager(gpu_ext):
    import torch.nn.functional as F
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.parallel.graph import GraphedStep
    m1, m2 = _mlp(1), _mlp(1)
    d1, d2 = DDP(m1, O.Adam(1e-2)), DDP(m2, O.Adam(1e-2))
    x = torch.randn(16, 32, device="cuda")
    y = torch.randn(16, 1, device="cuda")

    def loss_fn(d, xx, yy):
        return F.mse_loss(d(xx), yy)

    g = GraphedStep(d1, loss_fn, x, y, warmup=2)
    for _ in range(2):  # the warm-up steps GraphedStep ran eagerly (capture itself executes nothing)
        loss_fn(d2, x, y).backward()
        d2.step()
    assert d1.step_count == 2
    for _ in range(4):
        g(x, y)
        loss_fn(d2, x, y).backward()
        d2.step()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_bf16_master_weights(gpu_ext):
    """bf16 params + fp32 master/moments: the master tracks the fp32 reference closely."""
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    m = _mlp(2)
    ref = _mlp(2)
    m = m.bfloat16()
    ddp = DDP(m, O.Adam(1e-3))
    assert all(b.master is not None for b in ddp.buckets)
    ps = {n: p.detach().clone() for n, p in ref.named_parameters()}
    st = O.setup(O.Adam(1e-3), ps)
    x = torch.randn(16, 32, device="cuda")
    for _ in range(3):
        m(x.bfloat16()).float().sum().backward()
        grads = {n: p.grad.float().clone() for n, p in m.named_parameters()}
        ddp.step()
        st, ps = O.update(st, ps, grads)
    master = torch.cat([b.master for b in ddp.buckets])
    assert torch.isfinite(master).all()
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.float(), ps[n], rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("force_comm", [False, True])
def test_overlap_opt_bitwise_gpu(gpu_ext, force_comm):
    """Per-bucket optimiser overlap (updates enqueued from the backward hooks: on the RCCL stream
    behind each bucket's allreduce with force_comm, on a side stream at world 1) gives bit-identical
    parameters to the updates in step(), with bf16 parameters + fp32 masters, several buckets."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    FluxMPI.Init()
    x = torch.randn(64, 32, device="cuda").bfloat16()
    y = x.float().sum(1, keepdim=True).sin()
    outs = []
    for ov in (False, True):
        m = _mlp(3).bfloat16()
        d = DDP(m, O.Adam(1e-2), bucket_mb=0.004, first_bucket_mb=0.002, force_comm=force_comm, overlap_opt=ov,
                average=True)
        assert d.overlap_opt == ov and len(d.buckets) > 1
        for _ in range(4):
            ((d(x).float() - y) ** 2).mean().backward()
            d.step()
        torch.cuda.synchronize()
        outs.append([p.detach().clone() for p in m.parameters()] + [b.master.clone() for b in d.buckets])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
