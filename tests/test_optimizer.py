"""Mirror of reference test/test_optimizer.jl (DistributedOptimizer, allreduce_gradients)."""


def _state_equal(a, b):
    import torch
    if isinstance(a, torch.Tensor):
        return torch.equal(a, b)
    if isinstance(a, tuple):
        return len(a) == len(b) and all(_state_equal(x, y) for x, y in zip(a, b))
    return a == b


def worker():
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as Optimisers

    FluxMPI.Init(verbose=True)
    W = FluxMPI.total_workers()

    opt = Optimisers.Adam(0.001)
    ps = {"a": torch.zeros(4, dtype=torch.float64), "b": torch.zeros(4, dtype=torch.float64)}
    st_opt = Optimisers.setup(opt, ps)
    dopt = FluxMPI.DistributedOptimizer(opt)
    st_dopt = Optimisers.setup(dopt, ps)
    assert _state_equal(st_dopt["a"].state, st_opt["a"].state)
    assert _state_equal(st_dopt["b"].state, st_opt["b"].state)
    st_dopt = FluxMPI.synchronize(st_dopt, root_rank=0)

    gs = {"a": torch.ones(4, dtype=torch.float64), "b": torch.ones(4, dtype=torch.float64)}
    _, ps_dopt = Optimisers.update(st_dopt, ps, {k: v.clone() for k, v in gs.items()})
    _, ps_opt = Optimisers.update(st_opt, ps, {"a": gs["a"] * W, "b": gs["b"] * W})
    assert torch.allclose(ps_dopt["a"], ps_opt["a"], atol=1e-5, rtol=1e-5)
    assert torch.allclose(ps_dopt["b"], ps_opt["b"], atol=1e-5, rtol=1e-5)
    assert torch.equal(ps["a"], torch.zeros(4, dtype=torch.float64))  # `update` is out of place

    # SUM semantics checked with a rule that is NOT scale invariant (Descent)
    d = FluxMPI.DistributedOptimizer(Optimisers.Descent(0.5))
    st = Optimisers.setup(d, ps)
    _, p2 = Optimisers.update(st, ps, {"a": torch.ones(4, dtype=torch.float64), "b": torch.ones(4, dtype=torch.float64)})
    assert torch.equal(p2["a"], torch.full((4,), -0.5 * W, dtype=torch.float64))
    # average=True extension
    d = FluxMPI.DistributedOptimizer(Optimisers.Descent(0.5), average=True)
    st = Optimisers.setup(d, ps)
    _, p3 = Optimisers.update(st, ps, {"a": torch.ones(4, dtype=torch.float64), "b": torch.ones(4, dtype=torch.float64)})
    assert torch.allclose(p3["a"], torch.full((4,), -0.5, dtype=torch.float64))

    # allreduce_gradients
    gs = {"a": torch.ones(4), "b": torch.ones(4), "c": None, "n": (torch.ones(2, 2), "sym")}
    gs_ = FluxMPI.allreduce_gradients(gs, on_gpu=False)
    assert torch.equal(gs_["a"], torch.ones(4) * W)
    assert torch.equal(gs_["b"], torch.ones(4) * W)
    assert gs_["c"] is None and gs_["n"][1] == "sym"
    assert torch.equal(gs_["n"][0], torch.ones(2, 2) * W)
    FluxMPI.Finalize()


def test_optimizer(spmd):
    spmd("tests.test_optimizer:worker")


def worker_buckets():
    """Many leaves, tiny buckets: exercises the multi-bucket + direct paths of allreduce_tensors."""
    import os
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel.bucket import allreduce_tensors, broadcast_tensors

    FluxMPI.Init()
    W, r = FluxMPI.total_workers(), FluxMPI.local_rank()
    g = torch.Generator().manual_seed(0)
    shapes = [(3,), (17, 5), (1,), (1000,), (64, 64), (7, 7, 3), (5000,)]
    ts = [torch.randn(s, generator=g) * (r + 1) for s in shapes]
    expect = [t / (r + 1) * sum(range(1, W + 1)) for t in ts]
    allreduce_tensors(ts, "+", bucket_bytes=4096)
    for t, e in zip(ts, expect):
        assert torch.allclose(t, e, rtol=1e-5, atol=1e-5)
    bs = [torch.full(s, float(r)) for s in shapes] + [torch.full((4,), r, dtype=torch.int64)]
    broadcast_tensors(bs, root=W - 1, bucket_bytes=2048)
    for b in bs:
        assert torch.all(b == W - 1)
    FluxMPI.Finalize()


def test_bucketed_collectives(spmd):
    spmd("tests.test_optimizer:worker_buckets", nprocs=3)


def test_hyperparameters_cast_to_leaf_precision():
    """Optimisers.jl converts η, β, ϵ to ``eltype(x)`` (``T(η)``): bf16 / fp16 leaves see the
    rounded values. Parity unpinned against Julia itself (not installed);
    the expected numbers are the IEEE / bfloat16 roundings."""
    import torch
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.optimisers import _T

    bf, hf, f32, f64 = (torch.zeros(2, dtype=d) for d in (torch.bfloat16, torch.float16, torch.float32,
                                                           torch.float64))
    assert _T(bf, 0.9) == 0.8984375 and _T(bf, 0.999) == 1.0
    assert _T(hf, 0.9) == 0.89990234375 and _T(hf, 0.999) == 0.9990234375
    assert _T(hf, 1e-8) == 0.0  # below fp16's smallest subnormal, as Float16(1e-8) in Julia
    assert _T(f32, 0.1) == float(torch.tensor(0.1, dtype=torch.float32)) and _T(f64, 0.1) == 0.1
    st = O.setup(O.Adam(1e-3), {"a": hf, "b": f64})
    assert st["a"].state[2] == (0.89990234375, 0.9990234375)
    assert st["b"].state[2] == (0.9, 0.999)
    # one fp16 Adam step: the bias corrections use the rounded beta^t
    x = torch.ones(4, dtype=torch.float16)
    st = O.setup(O.Adam(0.5), x)
    g = torch.full((4,), 0.25, dtype=torch.float16)
    st, x2 = O.update(st, x, g)
    b1, b2 = 0.89990234375, 0.9990234375
    m, v = (1 - b1) * 0.25, (1 - b2) * 0.0625
    eps16 = float(torch.tensor(1e-7, dtype=torch.float16))  # Optimisers.jl _eps(Float16, 1e-8)
    step = m / (1 - b1) / ((v / (1 - b2)) ** 0.5 + eps16) * 0.5
    torch.testing.assert_close(x2.float(), torch.full((4,), 1.0 - step), rtol=2e-3, atol=2e-3)
    assert st.state[2] == (_T(x, b1 * b1), _T(x, b2 * b2))


def test_fp16_adam_zero_gradient_is_finite():
    """ϵ on fp16 leaves follows Optimisers.jl's ``_eps``: floored at Float16(1e-7), never 0, so
    an element whose gradient has always been zero stays put instead of becoming NaN
    (0 / (sqrt(0) + 0)); AdaGrad and RMSProp likewise. Eager and fused paths."""
    import torch
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.optimisers import _eps

    hf = torch.zeros(2, dtype=torch.float16)
    assert _eps(hf, 1e-8) == float(torch.tensor(1e-7, dtype=torch.float16)) > 0
    assert _eps(hf, 0.0) == 0.0 and _eps(hf, 1e-3) == float(torch.tensor(1e-3, dtype=torch.float16))
    assert _eps(torch.zeros(1, dtype=torch.bfloat16), 1e-8) == float(torch.tensor(1e-8, dtype=torch.bfloat16))
    for rule in (O.Adam(1e-3), O.AdaGrad(0.1), O.RMSProp(1e-3)):
        x = torch.ones(4, dtype=torch.float16)
        g = torch.tensor([0.5, 0.0, -0.25, 0.0], dtype=torch.float16)
        st = O.setup(rule, {"w": x})
        for _ in range(3):
            st, out = O.update(st, {"w": x}, {"w": g})
            x = out["w"]
        assert torch.isfinite(x).all(), (type(rule).__name__, x)
        assert x[1] == 1.0 and x[3] == 1.0, (type(rule).__name__, x)


def test_same_dense_layouts():
    """The fused-optimiser eligibility check on layouts (CPU tensors: the check itself)."""
    import torch
    from fluxmpi_amd.optimisers import _same_dense
    w = torch.zeros(8, 3, 7, 7).contiguous(memory_format=torch.channels_last)
    g = torch.zeros_like(w)
    assert _same_dense(w, g, torch.zeros_like(w), torch.zeros_like(w))
    assert not _same_dense(w, torch.zeros(8, 3, 7, 7))          # strides differ
    assert not _same_dense(torch.zeros(4, 6)[:, :3], torch.zeros(4, 3))  # gaps
    assert _same_dense(torch.nn.Parameter(torch.zeros(5, 5)), torch.zeros(5, 5))
