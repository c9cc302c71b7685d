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
        # the reference's tolerance (test/test_optimizer.jl:20-26): W-rank fp32 sums in another order
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-5)
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
    spmd("tests.test_ddp:worker_ddp")


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
    spmd("tests.test_ddp:worker_ddp_resnet")


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


def test_ddp_force_comm_world1_matches():
    """force_comm runs hooks + packing + (identity) collectives at world 1; same result."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    for grad_mode in ("steal", "view"):
        m1, m2 = _mlp(0), _mlp(0)
        d1 = DDP(m1, O.Adam(1e-2), bucket_mb=0.001, first_bucket_mb=0.0005, grad_mode=grad_mode, force_comm=True)
        d2 = DDP(m2, O.Adam(1e-2), bucket_mb=0.001, first_bucket_mb=0.0005, grad_mode=grad_mode)
        assert d1.communicate and d1._hooks and not d2.communicate and not d2._hooks
        x, y = _data(0)
        for _ in range(3):
            for d in (d1, d2):
                ((d(x) - y) ** 2).mean().backward()
            assert all(b.launched for b in d1.buckets)  # every bucket launched from the hooks
            d1.step()
            d2.step()
        for p, q in zip(m1.parameters(), m2.parameters()):
            assert torch.equal(p, q)
        assert d1.comm_summary()["comm"] != "none" and d2.comm_summary()["comm"] == "none"


def test_ddp_step_without_zero_grad_rearms():
    """step(zero_grad=False) must re-arm the buckets: the next step launches again."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    m = _mlp(0)
    d = DDP(m, O.Descent(0.1), bucket_mb=0.001, first_bucket_mb=0.0005, force_comm=True)
    x, y = _data(0)
    ((d(x) - y) ** 2).mean().backward()
    d.step(zero_grad=False)
    assert all(not b.launched and b.pending == len(b.params) for b in d.buckets) and d._next_launch == 0
    ((d(x) - y) ** 2).mean().backward()
    assert all(b.launched for b in d.buckets)
    d.step()


def worker_ddp_no_zero_grad():
    """``step(zero_grad=False)``: the next step applies the rank-sum of BOTH backwards'
    gradients, S1 + S2 (SUM) or (S1 + S2) / W (average) — not W*S1 + S2 (VERDICT r2 repro:
    Linear(4->1), x = rank+1, Descent(1.0) applied 9 instead of 6 at step 2)."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.utils.debug import check_replicas

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    S = float(sum(k + 1 for k in range(W)))  # the per-step rank-sum of d(sum(w.x))/dw
    for grad_mode in ("steal", "view"):
        for average in (False, True):
            for overlap in (True, False):
                m = torch.nn.Linear(4, 1, bias=False)
                with torch.no_grad():
                    m.weight.fill_(10.0)
                d = DDP(m, O.Descent(1.0), grad_mode=grad_mode, average=average, overlap=overlap)
                x = torch.full((1, 4), float(r + 1))
                scale = 1.0 / W if average else 1.0
                expect = 10.0
                # zero_grad pattern: F F T T -> applied S, 2S, 3S, S
                for k, zg in enumerate((False, False, True, True)):
                    d(x).sum().backward()
                    d.step(zero_grad=zg)
                    expect -= scale * S * (k + 1 if k < 3 else 1)
                    torch.testing.assert_close(m.weight.detach(), torch.full((1, 4), expect),
                                               msg=f"{grad_mode} avg={average} ov={overlap} step {k}")
                    check_replicas(m)
                # a step with no backward after step(zero_grad=False) applies the carried sum again
                d(x).sum().backward()
                d.step(zero_grad=False)
                expect -= scale * S
                d.step()
                expect -= scale * S
                torch.testing.assert_close(m.weight.detach(), torch.full((1, 4), expect))
    FluxMPI.Finalize()


def test_ddp_no_zero_grad_gloo(spmd):
    spmd("tests.test_ddp:worker_ddp_no_zero_grad", timeout=120)


def test_ddp_master_follows_outside_param_changes(tmp_path):
    """bf16 params with fp32 masters: load_state_dict / checkpoint.load / in-place edits made
    outside the engine are picked up at the next step."""
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.utils import checkpoint

    def bf16(seed):
        return _mlp(seed).to(torch.bfloat16)

    x, y = _data(0)
    x, y = x.bfloat16(), y.bfloat16()
    for how in ("load_state_dict", "checkpoint", "inplace"):
        m = bf16(0)
        d = DDP(m, O.Descent(0.1), master_weights=True)
        assert all(b.master is not None for b in d.buckets)
        src = bf16(1)
        if how == "load_state_dict":
            m.load_state_dict(src.state_dict())
        elif how == "checkpoint":
            checkpoint.save(str(tmp_path / "m.pt"), src)
            checkpoint.load(str(tmp_path / "m.pt"), like=m)
        else:
            with torch.no_grad():
                for p, q in zip(m.parameters(), src.parameters()):
                    p.copy_(q)
        # reference: a fresh engine built on the loaded weights
        m_ref = bf16(1)
        d_ref = DDP(m_ref, O.Descent(0.1), master_weights=True)
        for dd in (d, d_ref):
            ((dd(x) - y) ** 2).mean().backward()
            dd.step()
        for p, q in zip(m.parameters(), m_ref.parameters()):
            assert torch.equal(p, q), how
    # explicit refresh + a checkpoint without masters
    m = bf16(0)
    d = DDP(m, O.Adam(1e-2), master_weights=True)
    sd = d.state_dict()
    for b in sd["buckets"]:
        b["master"] = None
    with torch.no_grad():
        for p in m.parameters():
            p.zero_()
    sd["module"] = bf16(2).state_dict()
    d.load_state_dict(sd)
    for b in d.buckets:
        assert torch.equal(b.master, b.flat_param.float())
    d.refresh_master()


def test_ddp_optimiser_state_channels_last():
    """optimiser_state() views follow the parameter memory order (NHWC conv weights)."""
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(4, 2, 3))
    ref = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(4, 2, 3))
    ref.load_state_dict(net.state_dict())
    net = net.to(memory_format=torch.channels_last)
    assert net[0].weight.is_contiguous(memory_format=torch.channels_last)
    d = DDP(net, O.Adam(1e-2))
    ps = {n: p.detach().clone() for n, p in ref.named_parameters()}
    st = O.setup(O.Adam(1e-2), ps)
    x = torch.randn(2, 3, 6, 6)
    for _ in range(2):
        d(x.contiguous(memory_format=torch.channels_last)).square().mean().backward()
        d.step()
        for n, p in ref.named_parameters():
            p.data.copy_(ps[n])
            p.grad = None
        ref(x).square().mean().backward()
        st, ps = O.update(st, ps, {n: p.grad for n, p in ref.named_parameters()})
    state = d.optimiser_state()
    for n in ps:
        torch.testing.assert_close(state[n].state[0], st[n].state[0], rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(state[n].state[1], st[n].state[1], rtol=1e-4, atol=1e-9)


def worker_ddp_master_sync():
    """``synchronize`` of DDP-managed bf16 params must leave the fp32 masters
    identical on every rank — through the engine (``synchronize(model)``) and through a plain
    tensor tree (``synchronize(params)``), with small buckets so some leaves are "direct"
    (reduced/broadcast in place, no pack kernel)."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.utils.debug import check_replicas

    FluxMPI.Init()
    r = FluxMPI.local_rank()
    for how in ("module", "tree", "flux_model"):
        m = _mlp(3).to(torch.bfloat16)
        d = DDP(m, O.Adam(1e-2), master_weights=True, bucket_mb=0.0005, first_bucket_mb=0.0002)
        assert all(b.master is not None for b in d.buckets)
        # ranks drift apart (e.g. a rank-local edit): rank r's params move by r * 1e-2 + tiny
        with torch.no_grad():
            for p in m.parameters():
                p.add_(r * 1e-2 + 1e-4 * torch.randn_like(p))
        d.refresh_master()  # the edits are "known": only the synchronize below changes params
        with torch.no_grad():
            for b in d.buckets:  # and the masters hold bits the bf16 params cannot show
                for p, o in zip(b.params, b.offsets):
                    b.master[o:o + p.numel()] += 1e-5 * (r + 1)
        if how == "module":
            FluxMPI.synchronize(m)
        elif how == "flux_model":
            FluxMPI.synchronize(FluxMPI.FluxMPIFluxModel(m))
        else:
            FluxMPI.synchronize({n: p for n, p in m.named_parameters()})
        x, y = _data(r)
        for _ in range(3):
            ((d(x.bfloat16()) - y.bfloat16()) ** 2).mean().backward()
            d.step()
        check_replicas(m)
        for b in d.buckets:
            for p, o in zip(b.params, b.offsets):  # the slices (alignment padding is never used)
                g = FluxMPI.allgather(b.master[o:o + p.numel()].clone())
                assert torch.equal(g[0], g[1]), how
    FluxMPI.Finalize()


def test_ddp_master_sync_gloo(spmd):
    spmd("tests.test_ddp:worker_ddp_master_sync", timeout=120)


def worker_ddp_frozen_param_sync():
    """synchronize(model) of a DDP-managed model reaches the parameters outside every bucket
    (requires_grad=False: a frozen layer) as the reference's synchronize! reaches every leaf."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    r = FluxMPI.local_rank()
    model = _mlp(100 + r)  # different values per rank
    frozen = next(iter(model.parameters()))
    frozen.requires_grad_(False)
    d = DDP(model, O.Descent(0.1), force_comm=True)
    assert all(id(frozen) != id(p) for b in d.buckets for p in b.params)
    with torch.no_grad():
        frozen.fill_(float(r + 1))
    FluxMPI.synchronize(model, root_rank=0)
    g = FluxMPI.allgather(frozen.detach().clone())
    assert torch.equal(g[0], g[1]) and float(g[1].flatten()[0]) == 1.0
    FluxMPI.Finalize()


def test_ddp_frozen_param_sync_gloo(spmd):
    spmd("tests.test_ddp:worker_ddp_frozen_param_sync", timeout=120)


def test_engine_registry_does_not_keep_engines_alive():
    """The module -> engine registry holds the engine weakly: a discarded DDP is collected."""
    import gc
    import weakref

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP, engine_for

    FluxMPI.Init()
    model = _mlp(3)
    d = DDP(model, O.Descent(0.1))
    assert engine_for(model) is d
    ref = weakref.ref(d)
    del d
    gc.collect()
    assert ref() is None and engine_for(model) is None


def _opt_overlap_run(overlap_opt, rule_name, steps=3, rank=0, zero_grad_every=1):
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    rule = {"adam": O.Adam(1e-2), "momentum": O.Momentum(0.05, 0.9)}[rule_name]
    model = _mlp(7)
    ddp = DDP(model, rule, bucket_mb=0.001, first_bucket_mb=0.0005, overlap=True, overlap_opt=overlap_opt,
              average=True)
    assert ddp.overlap_opt == overlap_opt
    x, y = _data(rank)
    for s in range(steps):
        ((ddp(x) - y) ** 2).mean().backward()
        ddp.step(zero_grad=(s % zero_grad_every == 0))
    return [p.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("rule_name", ["adam", "momentum"])
def test_overlap_opt_world1_bitwise(rule_name):
    """Per-bucket updates enqueued from the backward hooks == updates in step(), bit for bit."""
    a = _opt_overlap_run(False, rule_name)
    b = _opt_overlap_run(True, rule_name)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def worker_overlap_opt():
    import fluxmpi_amd as FluxMPI
    FluxMPI.Init()
    r = FluxMPI.local_rank()
    for rule_name in ("adam", "momentum"):
        for zge in (1, 2):  # 2: step(zero_grad=False) every other step (the carried reduced sum)
            a = _opt_overlap_run(False, rule_name, steps=4, rank=r, zero_grad_every=zge)
            b = _opt_overlap_run(True, rule_name, steps=4, rank=r, zero_grad_every=zge)
            for x, y in zip(a, b):
                assert torch.equal(x, y), (rule_name, zge)
    FluxMPI.Finalize()


def test_overlap_opt_two_ranks_gloo(spmd):
    spmd("tests.test_ddp:worker_overlap_opt", timeout=180)


@pytest.mark.parametrize("how", ["overlap_opt", "force_comm"])
def test_second_backward_before_step_raises(how):
    """a second backward that reaches a bucket already reduced (and, with overlap_opt,
    already applied) before step() must fail loudly, not drop or corrupt the update; accumulation
    under no_sync() keeps working."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    kw = {"overlap_opt": True} if how == "overlap_opt" else {"force_comm": True, "overlap_opt": False}
    model = _mlp(5)
    d = DDP(model, O.Adam(1e-2), bucket_mb=0.001, first_bucket_mb=0.0005, overlap=True, **kw)
    x, y = _data(0)
    ((d(x) - y) ** 2).mean().backward()
    with pytest.raises(RuntimeError, match="second backward"):
        ((d(x) - y) ** 2).mean().backward()
    d.step()
    # the supported accumulation pattern still works after the error
    with d.no_sync():
        ((d(x[:4]) - y[:4]) ** 2).sum().backward()
    ((d(x[4:]) - y[4:]) ** 2).sum().backward()
    d.step()
    assert all(torch.isfinite(p).all() for p in model.parameters())
