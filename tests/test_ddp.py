"""The DDP engine (flat bucket views, hook-driven overlap, fused optimiser) on CPU/gloo."""
import pytest
import torch
import torch.nn.functional as F


def _mlp(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.Tanh(), torch.nn.Linear(16, 16), torch.nn.Tanh(),
                               torch.nn.Linear(16, 1))


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(8, 5, generator=g)
    return x, x.sum(1, keepdim=True) ** 2


@pytest.mark.parametrize("grad_mode", ["steal", "view"])
@pytest.mark.parametrize("rule_name", ["adam", "adamw", "descent", "momentum", "nesterov"])
def test_ddp_world1_matches_functional(rule_name, grad_mode):
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    def rule():
        return {"adam": O.Adam(1e-2), "adamw": O.AdamW(1e-2, decay=0.1), "descent": O.Descent(0.05),
                "momentum": O.Momentum(0.05, 0.9), "nesterov": O.Nesterov(0.05, 0.9)}[rule_name]

    m1, m2 = _mlp(0), _mlp(0)
    ddp = DDP(m1, rule(), bucket_mb=0.001, first_bucket_mb=0.0005, grad_mode=grad_mode)  # several tiny buckets
    assert len(ddp.buckets) > 1
    ps = {n: p.detach().clone() for n, p in m2.named_parameters()}
    st = O.setup(rule(), ps)
    x, y = _data(0)
    for _ in range(4):
        loss = ((ddp(x) - y) ** 2).mean()
        loss.backward()
        ddp.step()
        for n, p in m2.named_parameters():
            p.data.copy_(ps[n])
            p.grad = None
        ((m2(x) - y) ** 2).mean().backward()
        st, ps = O.update(st, ps, {n: p.grad for n, p in m2.named_parameters()})
    for n, p in m1.named_parameters():
        torch.testing.assert_close(p.detach(), ps[n], rtol=1e-5, atol=1e-6)
    if rule_name == "adam":
        leaf = ddp.optimiser_state()["0.weight"]
        torch.testing.assert_close(leaf.state[0], st["0.weight"].state[0], rtol=1e-4, atol=1e-6)


def worker_ddp():
    import fluxmpi_amd as FluxMPI

    FluxMPI.Init()
    for mode in ("steal", "view"):
        _ddp_checks(mode)
    FluxMPI.Finalize()


def _ddp_checks(grad_mode):
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    model = _mlp(1000 + r)  # different init per rank: DDP must broadcast rank 0's
    ddp = DDP(model, O.Descent(0.1), bucket_mb=0.001, first_bucket_mb=0.0005, overlap=True, grad_mode=grad_mode)
    ref = _mlp(1000)
    x, y = _data(r)
    for step in range(3):
        loss = ((ddp(x) - y) ** 2).mean()
        loss.backward()
        ddp.step()
        # reference: sum of every rank's gradient, applied with Descent
        ref.zero_grad()
        for k in range(W):
            xk, yk = _data(k)
            ((ref(xk) - yk) ** 2).mean().backward()
        with torch.no_grad():
            for p in ref.parameters():
                p -= 0.1 * p.grad
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
    # ranks hold identical parameters
    for p in model.parameters():
        g = FluxMPI.allgather(p.detach().clone())
        assert all(torch.equal(g[0], g[i]) for i in range(W))
    # gradient accumulation with no_sync: two half-batches == one full batch
    with ddp.no_sync():
        ((ddp(x[:4]) - y[:4]) ** 2).sum().backward()
    ((ddp(x[4:]) - y[4:]) ** 2).sum().backward()
    ddp.reduce_gradients()
    acc = [p.grad.clone() for p in model.parameters()]
    ddp.zero_grad()
    ((ddp(x) - y) ** 2).sum().backward()
    ddp.reduce_gradients()
    for a, p in zip(acc, model.parameters()):
        torch.testing.assert_close(a, p.grad, rtol=1e-5, atol=1e-5)
    ddp.step()

    # low-precision wire format (K5 cast): same result within bf16 rounding
    m_a, m_b = _mlp(7), _mlp(7)
    d_a = DDP(m_a, O.Descent(0.1), comm_dtype=torch.bfloat16, grad_mode=grad_mode)
    d_b = DDP(m_b, O.Descent(0.1), grad_mode=grad_mode)
    for d in (d_a, d_b):
        ((d(x) - y) ** 2).mean().backward()
        d.step()
    for p, q in zip(m_a.parameters(), m_b.parameters()):
        torch.testing.assert_close(p, q, rtol=2e-2, atol=2e-3)


def test_ddp_gloo(spmd):
    spmd("tests.test_ddp:worker_ddp", nprocs=2)


def worker_ddp_resnet():
    """The bench workload's shape on CPU/gloo: a bottleneck ResNet (fused-BN modules, hybrid
    conv config — both fall back to PyTorch on CPU) under DDP with hook-driven overlap across
    several buckets. Weak scaling: every rank has its own batch; the result must equal one
    process stepping with the sum of all ranks' gradients."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    torch.manual_seed(5)
    model = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused")
    ref = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused")
    ref.load_state_dict(model.state_dict())
    ddp = DDP(model, O.Descent(0.05), bucket_mb=0.5, first_bucket_mb=0.1, overlap=True)
    assert len(ddp.buckets) >= 3
    xs = [torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(10 + k)) for k in range(W)]
    ys = [torch.randint(0, 10, (4,), generator=torch.Generator().manual_seed(20 + k)) for k in range(W)]
    for _ in range(2):
        F.cross_entropy(ddp(xs[r]), ys[r]).backward()
        ddp.step()
        # reference: BN batch statistics are per rank (as in DDP), gradients summed over ranks
        ref.zero_grad()
        for k in range(W):
            F.cross_entropy(ref(xs[k]), ys[k]).backward()
        with torch.no_grad():
            for p in ref.parameters():
                p -= 0.05 * p.grad
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-4, atol=1e-5, msg=n)
    FluxMPI.Finalize()


def test_ddp_resnet_gloo(spmd):
    spmd("tests.test_ddp:worker_ddp_resnet", nprocs=2)


def test_bucket_launch_order_mixed_dtypes():
    """Buckets are ordered by when they complete (their last parameter in backward order):
    a small bucket of another dtype spread over the whole model goes last instead of
    blocking the in-order launches of every bucket after its first parameter."""
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    torch.manual_seed(0)
    layers = []
    for _ in range(6):
        layers += [torch.nn.Linear(64, 64), torch.nn.LayerNorm(64)]
    model = torch.nn.Sequential(*layers)
    for m in model:
        if isinstance(m, torch.nn.Linear):
            m.to(torch.float64)  # "bf16 weights": a different dtype from the norm parameters
    ddp = DDP(model, O.Descent(0.1), bucket_mb=0.05, first_bucket_mb=0.02)
    pos = {id(p): i for i, p in enumerate(reversed(list(model.parameters())))}
    last = [max(pos[id(p)] for p in b.params) for b in ddp.buckets]
    assert last == sorted(last)
    # the norm parameters' bucket completes with the first LayerNorm: behind every float64
    # bucket except the ones holding the first Linear (with the old first-parameter order
    # it came second and blocked all of them)
    kinds = [b.dtype for b in ddp.buckets]
    assert len(kinds) > 4 and kinds.index(torch.float32) >= len(kinds) - 3
