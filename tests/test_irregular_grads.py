"""SURVEY Q8 on the functional (reference-shaped) API: ranks whose gradient trees differ.

Reference behaviour (``src/optimizer.jl:20-23,45-65``): one collective per leaf that
has a gradient, so a rank with ``nothing`` for some leaf skips a collective the others
issue and the job hangs. Here the plan comes from the state / parameter tree and missing
gradients are zero-filled; a tree that genuinely differs raises CollectiveMismatchError.
"""
import torch


def _params():
    g = torch.Generator().manual_seed(3)
    return {"a": torch.randn(4, 3, generator=g), "b": torch.randn(5, generator=g), "c": torch.randn(2, 2, generator=g)}


def _grad(rank, name):
    g = torch.Generator().manual_seed(100 * rank + sum(map(ord, name)))
    return torch.randn(_params()[name].shape, generator=g)


def worker_irregular():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.utils.errors import CollectiveMismatchError

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()

    # 1. DistributedOptimizer: rank 1 has no gradient for "b" (DEQ-style irregular tree)
    ps = _params()
    st = O.setup(FluxMPI.DistributedOptimizer(O.Descent(0.1)), ps)
    grads = {n: _grad(r, n) for n in ps}
    if r == 1:
        grads["b"] = None
    st, ps = O.update_(st, ps, grads)
    ref = _params()
    for n in ref:
        total = sum(_grad(k, n) for k in range(W) if not (k == 1 and n == "b"))
        torch.testing.assert_close(ps[n], ref[n] - 0.1 * total)

    # same inside an OptimiserChain (the chain is collective because a member is)
    ps = _params()
    st = O.setup(O.OptimiserChain(FluxMPI.DistributedOptimizer(O.Descent(0.1)), O.WeightDecay(0.0)), ps)
    grads = {n: _grad(r, n) for n in ps}
    if r == 0:
        grads["c"] = None
    st, ps = O.update_(st, ps, grads)
    total_c = sum(_grad(k, "c") for k in range(1, W))
    torch.testing.assert_close(ps["c"], _params()["c"] - 0.1 * total_c)

    # 2. allreduce_gradients with the parameter tree: zero-filled sum
    grads = {n: _grad(r, n) for n in ps}
    if r == 1:
        grads["a"] = None
    out = FluxMPI.allreduce_gradients(grads, like=_params())
    torch.testing.assert_close(out["a"], sum(_grad(k, "a") for k in range(W) if k != 1))
    torch.testing.assert_close(out["b"], sum(_grad(k, "b") for k in range(W)))
    # a fresh `like` tree of the same structure (new object every step) skips the cross-rank
    # check on every rank; a gradient whose shape changed on one rank raises there instead of
    # entering a mismatched collective (the others are not sent into the collective either:
    # the same step raises the same way on the rank that differs, and we stop here)
    grads = {n: _grad(r, n) for n in ps}
    out = FluxMPI.allreduce_gradients(grads, like=_params())
    torch.testing.assert_close(out["c"], sum(_grad(k, "c") for k in range(W)))
    grads = {n: _grad(r, n) for n in ps}
    grads["c"] = torch.zeros(4) if r == 1 else grads["c"]
    if r == 1:
        try:
            FluxMPI.allreduce_gradients(grads, like=_params())
        except CollectiveMismatchError:
            pass
        else:
            raise AssertionError("a changed gradient shape did not raise")

    # 3. without `like`, differing trees raise instead of hanging (on every rank)
    grads = {n: _grad(r, n) for n in ps}
    if r == 1:
        grads["c"] = None
    try:
        FluxMPI.allreduce_gradients(grads)
    except CollectiveMismatchError:
        pass
    else:
        raise AssertionError("mismatched gradient trees did not raise")
    # and the group is still usable afterwards
    t = torch.ones(3)
    FluxMPI.allreduce(t, "+")
    assert torch.equal(t, torch.full((3,), float(W)))

    # 4. ADVICE r5: gradients in another dtype than their parameters (fp64 grads of fp32 params)
    # on the checked step; on a later step one of them is missing on EVERY rank — the zero fill
    # takes the checked plan's dtype, so a consistent run does not raise
    like = {"w": torch.zeros(3, 2), "v": torch.zeros(4)}
    out = FluxMPI.allreduce_gradients({"w": torch.ones(3, 2, dtype=torch.float64),
                                       "v": torch.ones(4, dtype=torch.float64)}, like=like)
    assert out["w"].dtype == torch.float64 and torch.equal(out["v"], torch.full((4,), float(W), dtype=torch.float64))
    out = FluxMPI.allreduce_gradients({"w": torch.ones(3, 2, dtype=torch.float64), "v": None}, like=like)
    assert out["v"].dtype == torch.float64 and torch.count_nonzero(out["v"]) == 0
    assert torch.equal(out["w"], torch.full((3, 2), float(W), dtype=torch.float64))
    FluxMPI.Finalize()


def test_irregular_gradient_trees(spmd):
    spmd("tests.test_irregular_grads:worker_irregular", timeout=120)


def test_zero_fill_only_for_collective_rules():
    """A local (non-collective) rule keeps Optimisers.jl's skip-on-nothing behaviour."""
    from fluxmpi_amd import optimisers as O
    ps = _params()
    st = O.setup(O.Momentum(0.1, 0.9), ps)
    st, ps2 = O.update_(st, ps, {"a": torch.ones(4, 3), "b": None, "c": None})
    assert torch.count_nonzero(st["b"].state) == 0
    torch.testing.assert_close(ps2["b"], _params()["b"])
