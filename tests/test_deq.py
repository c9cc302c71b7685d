"""DEQ model + Anderson solver ops (``csrc/kernels/anderson.hip``, ``fluxmpi_amd/ops/anderson.py``).

CPU: the solver converges to the fixed point of a contraction; the implicit-gradient DEQ
trains end to end. GPU: the HIP Gram / mix kernels against the plain fp32 PyTorch
composition of the same op.
"""
import pytest
import torch
import torch.nn.functional as F

from fluxmpi_amd.models.deq import anderson, deq_mnist
from fluxmpi_amd.ops import anderson as AO


def _ref_gram(X, Fv, n, last):
    G = (Fv[:, :n] - X[:, :n]).double()
    return torch.bmm(G, G.transpose(1, 2)), Fv[:, last].double().pow(2).sum(1)


def _ref_mix(X, Fv, alpha, beta):
    n = alpha.shape[1]
    a = alpha.double()[:, :, None]
    return beta * (a * Fv[:, :n].double()).sum(1) + (1 - beta) * (a * X[:, :n].double()).sum(1)


def test_anderson_contraction_cpu():
    torch.manual_seed(0)
    d = 64
    A = torch.randn(d, d)
    A = 0.5 * A / torch.linalg.matrix_norm(A, 2)
    b = torch.randn(3, d)
    f = lambda z: z @ A.T + b  # noqa: E731
    z, k, res = anderson(f, torch.zeros(3, d), max_iter=50, tol=1e-6)
    exact = torch.linalg.solve(torch.eye(d) - A, b.T).T
    assert res < 1e-4
    assert torch.allclose(z, exact, atol=1e-4), (z - exact).abs().max()
    assert 2 <= k < 50


def test_anderson_ops_fallback_cpu():
    torch.manual_seed(1)
    X, Fv = torch.randn(4, 5, 32), torch.randn(4, 5, 32)
    H, fn = AO.gram(X, Fv, 3, 2)
    Hr, fr = _ref_gram(X, Fv, 3, 2)
    assert torch.allclose(H.double(), Hr, rtol=1e-5, atol=1e-4) and torch.allclose(fn.double(), fr, rtol=1e-5)
    alpha = torch.randn(4, 3)
    want = _ref_mix(X.clone(), Fv, alpha, 0.7)
    z = AO.mix(X, Fv, alpha, 4, beta=0.7, z_dtype=torch.bfloat16)
    assert torch.allclose(X[:, 4].double(), want, rtol=1e-5, atol=1e-5)
    assert z.dtype == torch.bfloat16


def test_gram_solve_and_adjoint_step_fallback_cpu():
    """The CPU compositions behind AO.gram_solve / AO.adjoint_step (the GPU kernels' oracles)."""
    torch.manual_seed(2)
    bsz, m, d, n = 4, 5, 24, 3
    X = torch.randn(bsz, m, d)
    Fv = X + 0.1 * torch.randn(bsz, m, d)
    G = torch.zeros_like(X)
    alpha, res = AO.gram_solve(X, Fv, n, n - 1, G, tuple(range(n)), 1e-4, True)
    Hr, fr = _ref_gram(X, Fv, n, n - 1)
    A = torch.zeros(bsz, n + 1, n + 1, dtype=torch.float64)
    A[:, 0, 1:] = A[:, 1:, 0] = 1
    A[:, 1:, 1:] = Hr + 1e-4 * torch.eye(n, dtype=torch.float64)
    y = torch.zeros(bsz, n + 1, 1, dtype=torch.float64)
    y[:, 0] = 1
    torch.testing.assert_close(alpha.double(), torch.linalg.solve(A, y)[:, 1:, 0], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(res.double(), Hr[:, n - 1, n - 1].sum().sqrt() / (1e-5 + fr.sum().sqrt()),
                               rtol=1e-4, atol=1e-6)
    v, g, u = torch.randn(3, 2, 8, 4, 4).unbind(0)
    u_new, ss = AO.adjoint_step(v, g, u)
    torch.testing.assert_close(u_new, v + g)
    torch.testing.assert_close(ss, (v + g - u).pow(2).sum())


def test_deq_train_step_cpu():
    torch.manual_seed(2)
    model = deq_mnist(max_iter=12, bwd_iter=12)
    x, y = torch.randn(4, 1, 12, 12), torch.randint(0, 10, (4,))
    model.head = torch.nn.Linear(48 * 16, 10)
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    assert torch.isfinite(loss)
    g = model.deq.f.conv1.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("hdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("bsz,d", [(3, 36), (64, 4100), (256, 37632)])
def test_anderson_gram_gpu(n, bsz, d, fdt, hdt):
    """fdt bf16: the F history of a bf16 model; hdt bf16: its X history (FLUXMPI_DEQ_HIST=bf16).
    The reference reads the same bf16 values."""
    torch.manual_seed(n)
    m = max(n, 5)
    X = torch.randn(bsz, m, d, device="cuda").to(hdt)
    Fv = torch.randn(bsz, m, d, device="cuda").to(fdt)
    last = n - 1
    H, fn = AO.gram(X, Fv, n, last)
    Hr, fr = _ref_gram(X.float(), Fv.float(), n, last)
    torch.testing.assert_close(H.double(), Hr, rtol=1e-4, atol=1e-3 * d ** 0.5)
    torch.testing.assert_close(fn.double(), fr, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("hdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,beta", [(1, 1.0), (3, 1.0), (5, 1.0), (5, 0.8), (8, 0.5)])
@pytest.mark.parametrize("zdt", [None, torch.bfloat16, torch.float16])
def test_anderson_mix_gpu(n, beta, zdt, fdt, hdt):
    torch.manual_seed(10 + n)
    bsz, m, d = 37, 8, 4100
    X = torch.randn(bsz, m, d, device="cuda").to(hdt)
    Fv = torch.randn(bsz, m, d, device="cuda").to(fdt)
    alpha = torch.randn(bsz, n, device="cuda")
    slot = (n + 2) % m
    keep = X.clone()
    want = _ref_mix(X.float(), Fv.float(), alpha, beta)
    z = AO.mix(X, Fv, alpha, slot, beta, zdt)
    if hdt == torch.float32:
        torch.testing.assert_close(X[:, slot].double(), want, rtol=1e-5, atol=1e-4)
    else:  # the new iterate rounded to bf16 once
        torch.testing.assert_close(X[:, slot].double(), want, rtol=8e-3, atol=1e-3)
    others = [i for i in range(m) if i != slot]
    assert torch.equal(X[:, others], keep[:, others])
    if zdt is not None:
        assert z.dtype == zdt and z.shape == (bsz, d)
        if hdt == torch.float32:
            torch.testing.assert_close(z.float(), X[:, slot].to(zdt).float())
        else:  # z is the fp32 mix rounded to zdt, X[:, slot] the same value rounded to bf16
            torch.testing.assert_close(z.double(), want, rtol=8e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("bsz", [3, 256, 1000])
def test_anderson_gram_solve_gpu(n, bsz):
    """One-launch residual + pivoted (n+1)^2 solve (anderson_solve) vs the fp64 composition."""
    torch.manual_seed(20 + n)
    m, d = max(n, 5), 4100
    X = torch.randn(bsz, m, d, device="cuda")
    Fv = X + 0.1 * torch.randn(bsz, m, d, device="cuda")
    G = torch.zeros_like(X)
    last = n - 1
    lam = 1e-4
    alpha, res = AO.gram_solve(X, Fv, n, last, G, tuple(range(n)), lam, True)
    Hr, fr = _ref_gram(X, Fv, n, last)
    A = torch.zeros(bsz, n + 1, n + 1, dtype=torch.float64, device="cuda")
    A[:, 0, 1:] = A[:, 1:, 0] = 1
    A[:, 1:, 1:] = Hr + lam * torch.eye(n, dtype=torch.float64, device="cuda")
    y = torch.zeros(bsz, n + 1, 1, dtype=torch.float64, device="cuda")
    y[:, 0] = 1
    want = torch.linalg.solve(A, y)[:, 1:, 0]
    assert alpha.shape == (bsz, n) and alpha.dtype == torch.float32
    torch.testing.assert_close(alpha.double(), want, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(alpha.double().sum(1), torch.ones(bsz, dtype=torch.float64, device="cuda"),
                               rtol=1e-4, atol=1e-4)
    res_ref = Hr[:, last, last].sum().sqrt() / (1e-5 + fr.sum().sqrt())
    torch.testing.assert_close(res.double(), res_ref, rtol=1e-4, atol=1e-6)
    # no residual requested: same alpha, res None
    alpha2, res2 = AO.gram_solve(X, Fv, n, last, G, (last,), lam, False)
    assert res2 is None
    torch.testing.assert_close(alpha2, alpha, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cl", [False, True])
def test_adjoint_step_gpu(dtype, cl):
    """u_new = vjp + grad and |u_new - u|^2 in one pass vs the PyTorch composition."""
    torch.manual_seed(4)
    mf = torch.channels_last if cl else torch.contiguous_format
    v, g, u = (torch.randn(6, 48, 28, 28, device="cuda").to(dtype).contiguous(memory_format=mf) for _ in range(3))
    u_new, ss = AO.adjoint_step(v, g, u)
    want = v + g
    assert u_new.stride() == want.stride()
    torch.testing.assert_close(u_new, want, rtol=0, atol=0)
    ref = (want.float() - u.float()).pow(2).sum()
    torch.testing.assert_close(ss, ref, rtol=1e-4, atol=1e-3)
    # the convergence flag in the reduce's launch: flag = ss <= thresh2
    for scale, want_flag in ((1.01, 1.0), (0.99, 0.0)):
        flag = torch.full((1,), -1.0, device="cuda")
        t2 = (ref * scale).float()
        u2, ss2 = AO.adjoint_step(v, g, u, thresh2=t2, flag=flag)
        torch.testing.assert_close(u2, want, rtol=0, atol=0)
        torch.testing.assert_close(ss2, ref, rtol=1e-4, atol=1e-3)
        assert float(flag) == want_flag, (scale, float(flag))


@pytest.mark.gpu
def test_anderson_solver_gpu_matches_cpu():
    torch.manual_seed(3)
    d = 256
    A = torch.randn(d, d, dtype=torch.float64)
    A = (0.6 * A / torch.linalg.matrix_norm(A, 2)).float()
    b = torch.randn(16, d)
    zc, kc, _ = anderson(lambda z: z @ A.T + b, torch.zeros(16, d), max_iter=40, tol=1e-5)
    Ag, bg = A.cuda(), b.cuda()
    zg, kg, rg = anderson(lambda z: z @ Ag.T + bg, torch.zeros(16, d, device="cuda"), max_iter=40, tol=1e-5)
    assert rg < 1e-5 and abs(kg - kc) <= 2
    torch.testing.assert_close(zg.cpu(), zc, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("add,relu", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,groups", [((4, 48, 28, 28), 8), ((3, 16, 5, 7), 4), ((2, 64, 9, 9), 64)])
def test_fused_groupnorm_gpu(add, relu, dtype, shape, groups):
    from fluxmpi_amd.ops.groupnorm import FusedGroupNorm, _GroupNormFn  # noqa: F401

    torch.manual_seed(7)
    N, C, H, W = shape
    gn = FusedGroupNorm(groups, C).cuda()
    with torch.no_grad():
        gn.weight.normal_(1, 0.3)
        gn.bias.normal_(0, 0.3)
    cl = torch.channels_last
    x = (torch.randn(shape, device="cuda") + 0.3).to(dtype).contiguous(memory_format=cl).requires_grad_()
    a = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=cl).requires_grad_() if add else None
    y = gn(x, add=a, relu=relu)
    dy = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=cl)
    y.backward(dy)
    # fp32 PyTorch reference on the same (rounded) inputs
    xr = x.detach().float().clone().requires_grad_()
    ar = a.detach().float().clone().requires_grad_() if add else None
    wr = gn.weight.detach().clone().requires_grad_()
    br = gn.bias.detach().clone().requires_grad_()
    h = xr + ar if add else xr
    if relu:
        h = torch.relu(h)
    h = h.to(dtype).float()  # the kernel normalises the stored (rounded) h
    yr = torch.nn.functional.group_norm(h, groups, wr, br, gn.eps)
    yr.backward(dy.float())
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    if add:
        torch.testing.assert_close(a.grad.float(), ar.grad, **tol)
    gtol = dict(rtol=2e-2, atol=2e-2 * N * H * W ** 0.5) if dtype == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(gn.weight.grad, wr.grad, **gtol)
    torch.testing.assert_close(gn.bias.grad, br.grad, **gtol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_groupnorm_out_slot_gpu(gpu_ext, dtype):
    """gn_fwd_raw writing straight into strided history rows (the DEQ-CIFAR cell's last GroupNorm
    into its Anderson F slot): the dense output's values, the other rows untouched."""
    from fluxmpi_amd.ops.groupnorm import gn_fwd_raw
    torch.manual_seed(8)
    cl = torch.channels_last
    N, C, H, W = 4, 64, 9, 7
    x = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=cl)
    a = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=cl)
    w, b = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    y, *_ = gn_fwd_raw(x, a, w, b, 16, 1e-5, True)
    hist = torch.full((N, 3, C * H * W), float("nan"), device="cuda", dtype=dtype)
    ys, *_ = gn_fwd_raw(x, a, w, b, 16, 1e-5, True, out=hist[:, 1])
    assert ys.data_ptr() == hist[:, 1].data_ptr()
    torch.testing.assert_close(hist[:, 1], y.permute(0, 2, 3, 1).reshape(N, -1), rtol=0, atol=0)
    assert torch.isnan(hist[:, 0].float()).all() and torch.isnan(hist[:, 2].float()).all()


@pytest.mark.gpu
def test_deq_cell_fused_path_gpu():
    """The DEQ cell on channels_last bf16 takes the HIP GroupNorm path and matches the fp32 composition."""
    from fluxmpi_amd.models.deq import ResidualCell

    torch.manual_seed(8)
    cell = ResidualCell(48).cuda()
    z = torch.randn(8, 48, 14, 14, device="cuda").contiguous(memory_format=torch.channels_last)
    x = torch.randn_like(z)
    out = cell(z, x)
    n1, n2, n3 = cell.n1, cell.n2, cell.n3
    gn = lambda m, t: torch.nn.functional.group_norm(t, m.num_groups, m.weight, m.bias, m.eps)  # noqa: E731
    ref = gn(n3, torch.relu(z + gn(n2, x + cell.conv2(gn(n1, torch.relu(cell.conv1(z)))))))
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_deq_train_step_gpu_param_grads():
    """bf16 channels_last DEQ step on the GPU: every parameter (incl. the fused GroupNorms,
    whose reductions are skipped only inside the adjoint VJPs) gets a finite gradient."""
    torch.manual_seed(9)
    model = deq_mnist(max_iter=10, bwd_iter=10).cuda().to(memory_format=torch.channels_last)
    for m in model.modules():
        if not isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    x = torch.randn(16, 1, 28, 28, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    loss = F.cross_entropy(model(x).float(), y)
    loss.backward()
    assert torch.isfinite(loss)
    for name, p in model.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad.float()).all(), name
    assert model.deq.f.n3.weight.grad.abs().sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("hdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [2, 5, 8])
def test_anderson_gram_stored_g_gpu(n, fdt, hdt):
    """hdt bf16: X and the stored G = F - X rows in bf16 (G rounded once when stored; the fresh
    row's products use its exact fp32 difference)."""
    torch.manual_seed(20 + n)
    bsz, m, d = 64, 8, 4100
    X = torch.randn(bsz, m, d, device="cuda").to(hdt)
    Fv = torch.randn(bsz, m, d, device="cuda").to(fdt)
    G = torch.zeros_like(X)
    exact = hdt == torch.float32
    tol = dict(rtol=1e-4, atol=1e-3 * d ** 0.5) if exact else dict(rtol=1e-2, atol=2e-2 * d ** 0.5)
    H0, _ = AO.gram(X, Fv, n, n - 1, G, tuple(range(n)))  # all rows fresh: fills G
    torch.testing.assert_close(G[:, :n], (Fv[:, :n].float() - X[:, :n].float()).to(hdt))
    s = n // 2  # one row changes (the newest, `last`): only it is recomputed, the others come from G
    X[:, s].normal_()
    Fv[:, s].normal_()
    H, fn = AO.gram(X, Fv, n, s, G, (s,))
    Hr, fr = _ref_gram(X.float(), Fv.float(), n, s)
    torch.testing.assert_close(H.double(), Hr, **tol)
    torch.testing.assert_close(fn.double(), fr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(G[:, s], (Fv[:, s].float() - X[:, s].float()).to(hdt))
    # a fresh row that is not `last`: every row is recomputed from F - X (same result)
    t = (s + 1) % n
    X[:, t].normal_()
    H2, fn2 = AO.gram(X, Fv, n, s, G, (t,))
    Hr2, fr2 = _ref_gram(X.float(), Fv.float(), n, s)
    torch.testing.assert_close(H2.double(), Hr2, **tol)
    torch.testing.assert_close(fn2.double(), fr2, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("lag", [1, 2, 3])
def test_anderson_lagged_check_gpu(lag):
    """Lagged (no queue drain) convergence tests: at most `lag` extra iterations, same fixed point."""
    torch.manual_seed(3)
    d = 256
    A = torch.randn(d, d, dtype=torch.float64)
    A = (0.6 * A / torch.linalg.matrix_norm(A, 2)).float()
    b = torch.randn(16, d)
    zc, kc, _ = anderson(lambda z: z @ A.T + b, torch.zeros(16, d), max_iter=40, tol=1e-5)
    Ag, bg = A.cuda(), b.cuda()
    zg, kg, rg = anderson(lambda z: z @ Ag.T + bg, torch.zeros(16, d, device="cuda"), max_iter=40, tol=1e-5,
                          check_lag=lag)
    assert float(rg) < 1e-5 and kc - 2 <= kg <= kc + lag + 2
    torch.testing.assert_close(zg.cpu(), zc, rtol=1e-4, atol=1e-4)
    # not converging within max_iter: the residual stays on the device (no sync)
    z2, k2, r2 = anderson(lambda z: z @ Ag.T + bg, torch.zeros(16, d, device="cuda"), max_iter=4, tol=1e-12,
                          check_lag=lag)
    assert isinstance(r2, torch.Tensor) and r2.is_cuda and k2 == 3


@pytest.mark.gpu
def test_deq_lagged_matches_sync():
    """DEQ forward + implicit backward with lagged checks vs synchronous checks."""
    from fluxmpi_amd.models.deq import deq_mnist
    torch.backends.cudnn.deterministic = True  # MIOpen's default solvers vary run to run
    torch.manual_seed(0)
    # tight tolerances: both solves converge, so the lagged run's extra iterations change little
    kw = dict(max_iter=80, tol=1e-6, bwd_iter=80, bwd_tol=1e-6, restart=0)  # restarts depend on when a test is read
    m0 = deq_mnist(check_lag=0, **kw).cuda()
    m2 = deq_mnist(check_lag=2, **kw).cuda()
    m2.load_state_dict(m0.state_dict())
    x = torch.randn(8, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    outs = []
    for m in (m0, m2):
        out = m(x)
        torch.nn.functional.cross_entropy(out, y).backward()
        outs.append(out.detach())
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-3, atol=1e-3)
    for (n, p), q in zip(m0.named_parameters(), m2.parameters()):
        # the lagged solve runs up to 2 more (contracting) iterations: differences at the solver tolerance
        tol = 1e-3 * float(p.grad.abs().max()) + 1e-6
        torch.testing.assert_close(p.grad, q.grad, rtol=2e-2, atol=tol, msg=lambda m: f"{n}: {m}")
    assert m0.deq.last_bwd_iters < 80 and m2.deq.last_bwd_iters <= m0.deq.last_bwd_iters + 2
    assert m0.deq.last_iters < 79 and m2.deq.last_iters <= m0.deq.last_iters + 2


@pytest.mark.gpu
def test_deq_manual_vjp_matches_autograd(gpu_ext):
    """The adjoint's direct-kernel VJP (ResidualCell.forward_state / vjp) equals autograd's
    J^T u through the same cell (bf16 channels_last, 48 channels, MNIST-sized)."""
    from fluxmpi_amd.models.deq import ResidualCell
    from fluxmpi_amd.ops.groupnorm import skip_param_grads
    torch.manual_seed(0)
    cell = ResidualCell(48).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for p in cell.parameters():
            p.add_(0.05 * torch.randn_like(p))
    z = torch.randn(8, 48, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x = torch.randn_like(z)
    assert cell.manual_ok(z)
    out, state = cell.forward_state(z, x)
    z0 = z.clone().requires_grad_()
    f0 = cell(z0, x)
    # the fused cell kernel and the module path reduce the GroupNorm statistics in different
    # orders: equal to within one bf16 rounding of the output (2^-8 relative)
    torch.testing.assert_close(out.float(), f0.detach().float(), rtol=8e-3, atol=1e-2)
    for _ in range(2):
        u = torch.randn_like(z)
        with skip_param_grads():
            ref = torch.autograd.grad(f0, z0, u, retain_graph=True)[0]
        got = cell.vjp(state, u)
        rel = float((got.float() - ref.float()).norm() / ref.float().norm())
        assert rel < 1e-2, rel


@pytest.mark.gpu
def test_deq_train_step_manual_vjp_gpu(gpu_ext, monkeypatch):
    """A DEQ training step with the manual adjoint gives the same parameter gradients as the
    autograd adjoint."""
    import fluxmpi_amd.models.deq as D
    torch.manual_seed(1)
    grads = []
    for manual in (True, False):
        monkeypatch.setattr(D, "MANUAL_VJP", manual)
        torch.manual_seed(1)
        # the adjoint solved to 1e-4 (both variants then agree to the tolerance below; the bench
        # defaults, DEQ_MNIST_SOLVER, stop at 1e-2)
        m = deq_mnist(tol=1e-4, bwd_tol=1e-4).cuda().to(memory_format=torch.channels_last)
        for mod in m.modules():
            if type(mod).__name__ not in ("FusedBatchNorm2d",):
                for p in mod.parameters(recurse=False):
                    p.data = p.data.to(torch.bfloat16)
        x = torch.randn(16, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), device="cuda")
        F.cross_entropy(m(x).float(), y).backward()
        grads.append([p.grad.float().clone() for p in m.parameters()])
    # the two variants reach different bf16 fixed points (the fused cell and the module GroupNorms
    # round in different orders; the solve floors at ~2e-4 in bf16) and the adjoint amplifies that
    # by ~1 / (1 - rho): agreement to a few per cent (3-5 % measured), no parameter far off
    rels = [float((a - b).norm() / b.norm().clamp_min(1e-12)) for a, b in zip(*grads)]
    assert max(rels) < 1e-1 and sorted(rels)[len(rels) // 2] < 6e-2, rels


def _deq_bf16(**kw):
    kw.setdefault("restart", 0)  # exact eager / graphed comparisons: no stall-dependent restarts
    m = deq_mnist(**kw).cuda().to(memory_format=torch.channels_last)
    for mod in m.modules():
        if type(mod).__name__ not in ("FusedBatchNorm2d",):
            for p in mod.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    return m


def _graphed_vs_eager(steps, **kw):
    """``steps`` SGD training steps of the same bf16 DEQ, solver graphs off / on; per step the
    output, the parameter gradients and the iteration counts."""
    torch.manual_seed(7)
    x = torch.randn(32, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    runs = []
    for graphs in (False, True):
        torch.manual_seed(3)
        m = _deq_bf16(**kw)
        m.deq.use_graphs = graphs
        rec = []
        for step in range(steps):
            out = m(x)
            F.cross_entropy(out.float(), y).backward()
            rec.append((out.detach().float().clone(), [p.grad.float().clone() for p in m.parameters()],
                        m.deq.last_iters, m.deq.last_bwd_iters))
            # parameters change in place between steps (the same change in both runs, independent of
            # the gradients): the graphs must read the current weights / affine copies / filters
            with torch.no_grad():
                for i, p in enumerate(m.parameters()):
                    p.grad = None
                    p.mul_(1.0 + 0.03 * ((i + step) % 3 - 1))
        runs.append(rec)
        if graphs:
            gs = [g for g in m.deq._graphs.values() if g is not None]
            assert len(gs) == 1 and gs[0].g_fwd is not None and gs[0].g_adj is not None
    return runs


@pytest.mark.gpu
def test_deq_solver_graphs_match_eager(gpu_ext):
    """The solver graphs (deq.SolverGraphs) replay exactly the eager loops' launches: with no
    early exit (tol 0) four training steps — eager, capture, replay, replay — give the eager
    run's outputs, gradients and iteration counts (max_iter 13 / bwd_iter 12 also exercise the
    eager head and tail around the replayed periods)."""
    eager, graphed = _graphed_vs_eager(4, max_iter=13, tol=0.0, bwd_iter=12, bwd_tol=0.0)
    for s, ((oa, ga, ia, ba), (ob, gb, ib, bb)) in enumerate(zip(eager, graphed)):
        assert (ia, ba) == (ib, bb) == (12, 12), (s, ia, ba, ib, bb)
        torch.testing.assert_close(ob, oa, rtol=2e-2, atol=2e-2)
        for a, b in zip(ga, gb):
            rel = float((b - a).norm() / a.norm().clamp_min(1e-12))
            assert rel < 2e-2, (s, rel)


@pytest.mark.gpu
def test_deq_anderson_adjoint_graphs_match_eager(gpu_ext):
    """The Anderson adjoint (bwd_m = 5) through its own history and period graph
    (SolverGraphs.adjoint_anderson) replays the eager Anderson adjoint: same iteration counts,
    outputs and gradients over four training steps (eager, capture, replay, replay)."""
    eager, graphed = _graphed_vs_eager(4, max_iter=13, tol=0.0, bwd_iter=17, bwd_tol=0.0, bwd_m=5)
    for s, ((oa, ga, ia, ba), (ob, gb, ib, bb)) in enumerate(zip(eager, graphed)):
        assert (ia, ba) == (ib, bb) and ba >= 15, (s, ia, ba, ib, bb)
        torch.testing.assert_close(ob, oa, rtol=2e-2, atol=2e-2)
        for a, b in zip(ga, gb):
            rel = float((b - a).norm() / a.norm().clamp_min(1e-12))
            assert rel < 2e-2, (s, rel)


@pytest.mark.gpu
def test_deq_anderson_adjoint_gpu_matches_fixed_point(gpu_ext):
    """bf16 DEQ on the fused GPU path: gradients from the Anderson adjoint (bwd_tol 1e-3) agree
    with the fixed-point adjoint solved to 1e-4 within the bf16 fixed-point spread of
    test_deq_train_step_manual_vjp_gpu, in fewer iterations."""
    torch.manual_seed(5)
    x = torch.randn(32, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    grads, iters = [], []
    for bwd_m, bwd_tol in ((0, 1e-4), (5, 1e-3)):
        torch.manual_seed(3)
        m = _deq_bf16(tol=1e-4, max_iter=60, bwd_tol=bwd_tol, bwd_iter=120, bwd_m=bwd_m)
        for _ in range(3):  # eager, capture, replay: the last step's gradients are compared
            for p in m.parameters():
                p.grad = None
            F.cross_entropy(m(x).float(), y).backward()
        grads.append([p.grad.float().clone() for p in m.parameters()])
        iters.append(m.deq.last_bwd_iters)
    rels = [float((b - a).norm() / a.norm().clamp_min(1e-12)) for a, b in zip(*grads)]
    assert max(rels) < 1e-1 and sorted(rels)[len(rels) // 2] < 6e-2, rels
    assert iters[1] < iters[0], iters


@pytest.mark.gpu
def test_deq_solver_graphs_two_forwards_one_backward(gpu_ext):
    """loss = f(x1) + f(x2) at one shape: the second graphed forward overwrites the solver graphs'
    static state before the first call's adjoint runs, so that adjoint must run on its own state
    (generation check, deq.SolverGraphs.forward_state): graphed gradients == eager gradients."""
    torch.manual_seed(11)
    x1 = torch.randn(16, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x2 = torch.randn(16, 1, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    grads = []
    for graphs in (False, True):
        torch.manual_seed(3)
        m = _deq_bf16(max_iter=13, tol=0.0, bwd_iter=12, bwd_tol=0.0)
        m.deq.use_graphs = graphs
        for _ in range(2):  # eager first call, then capture: the third call replays
            F.cross_entropy(m(x1).float(), y).backward()
            for p in m.parameters():
                p.grad = None
        loss = F.cross_entropy(m(x1).float(), y) + F.cross_entropy(m(x2).float(), y)
        loss.backward()
        grads.append([p.grad.float().clone() for p in m.parameters()])
    for a, b in zip(*grads):
        rel = float((b - a).norm() / a.norm().clamp_min(1e-12))
        assert rel < 2e-2, rel


@pytest.mark.gpu
def test_deq_solver_graphs_early_exit(gpu_ext):
    """With a reachable tolerance the graphed solves stop within two periods of the eager ones
    (per-period, one-period-late tests) and land on the same fixed point."""
    eager, graphed = _graphed_vs_eager(3, max_iter=60, tol=1e-2, bwd_iter=60, bwd_tol=1e-2)
    for (oa, ga, ia, ba), (ob, gb, ib, bb) in zip(eager, graphed):
        assert ia < 59 and ba < 60, (ia, ba)  # the eager solves converge
        assert ia <= ib <= ia + 10 and ba <= bb <= ba + 10, (ia, ib, ba, bb)
        torch.testing.assert_close(ob, oa, rtol=5e-2, atol=5e-2)
        for a, b in zip(ga, gb):
            rel = float((b - a).norm() / a.norm().clamp_min(1e-12))
            assert rel < 2.5e-1, rel  # more (still contracting) iterations: a different point


def _cell_inputs(n=6, seed=0):
    from fluxmpi_amd.models.deq import ResidualCell
    torch.manual_seed(seed)
    cell = ResidualCell(48).cuda()
    with torch.no_grad():
        for p in cell.parameters():
            p.add_(0.05 * torch.randn_like(p))
        for c in (cell.conv1, cell.conv2):
            c.weight.mul_(20.0)  # O(1) activations through the convolutions
    cell = cell.to(torch.bfloat16).to(memory_format=torch.channels_last)
    z = torch.randn(n, 48, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x = torch.randn_like(z)
    return cell, z, x


def _ref_cell_fp32(cell, z, x):
    """f(z, x) in plain fp32 PyTorch ops from the cell's (bf16) parameters."""
    P = {k: v.float() for k, v in cell.state_dict().items()}

    def gn(t, i):
        m = getattr(cell, f"n{i}")
        return F.group_norm(t, m.num_groups, P[f"n{i}.weight"], P[f"n{i}.bias"], m.eps)

    zf, xf = z.float(), x.float()
    a1 = gn(torch.relu(F.conv2d(zf, P["conv1.weight"], padding=1)), 1)
    a2 = gn(F.conv2d(a1, P["conv2.weight"], padding=1) + xf, 2)
    return gn(torch.relu(zf + a2), 3)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.gpu
def test_deq_fused_cell_forward(gpu_ext, monkeypatch):
    """The one-kernel cell (ops/deq_cell.py) against the 5-launch raw path and an fp32 reference:
    output, saved GroupNorm inputs and statistics; the fp32 history-slot output."""
    from fluxmpi_amd.ops import deq_cell
    cell, z, x = _cell_inputs()
    assert deq_cell.supported(cell, z)
    out_f, st_f = cell.forward_state(z, x)
    monkeypatch.setattr(deq_cell, "ENABLED", False)
    out_u, st_u = cell.forward_state(z, x)
    ref = _ref_cell_fp32(cell, z, x)
    e_f, e_u = _rel(out_f, ref), _rel(out_u, ref)
    assert e_f < 2 * e_u + 5e-3, (e_f, e_u)
    assert _rel(out_f, out_u) < 2e-2
    for (hf, mf, rf, _), (hu, mu, ru, _) in zip(st_f[1:], st_u[1:]):
        assert _rel(hf, hu) < 2e-2 and _rel(mf, mu) < 2e-2 and _rel(rf, ru) < 2e-2
    # fp32 output into strided history rows (an Anderson slot): exactly the bf16 output's values
    monkeypatch.setattr(deq_cell, "ENABLED", True)
    n = z.shape[0]
    hist = torch.full((n, 3, z[0].numel()), float("nan"), device="cuda")
    deq_cell.cell_forward(cell, z, x, out32=hist[:, 1], want_out=False)
    torch.testing.assert_close(hist[:, 1], out_f.permute(0, 2, 3, 1).reshape(n, -1).float(), rtol=0, atol=0)
    assert torch.isnan(hist[:, 0]).all() and torch.isnan(hist[:, 2]).all()
    # bf16 output straight into a strided bf16 history slot (the bf16 F history)
    histb = torch.full((n, 3, z[0].numel()), float("nan"), device="cuda", dtype=torch.bfloat16)
    ob = deq_cell.cell_forward(cell, z, x, out_slot=histb[:, 1])
    assert ob.data_ptr() == histb[:, 1].data_ptr()
    torch.testing.assert_close(histb[:, 1], out_f.permute(0, 2, 3, 1).reshape(n, -1), rtol=0, atol=0)
    assert torch.isnan(histb[:, 0].float()).all() and torch.isnan(histb[:, 2].float()).all()


@pytest.mark.gpu
def test_deq_fused_cell_vjp(gpu_ext, monkeypatch):
    """The one-kernel adjoint VJP against the 5-launch raw VJP (same state) and fp32 autograd."""
    from fluxmpi_amd.ops import deq_cell
    cell, z, x = _cell_inputs(seed=1)
    _, state = cell.forward_state(z, x)
    zf = z.float().requires_grad_()
    ref_out = _ref_cell_fp32(cell, zf, x)
    for k in range(2):
        u = torch.randn_like(z)
        got = cell.vjp(state, u)
        monkeypatch.setattr(deq_cell, "ENABLED", False)
        base = cell.vjp(state, u)
        monkeypatch.setattr(deq_cell, "ENABLED", True)
        ref = torch.autograd.grad(ref_out, zf, u.float(), retain_graph=True)[0]
        e_f, e_u = _rel(got, ref), _rel(base, ref)
        assert e_f < 2 * e_u + 5e-3, (k, e_f, e_u)
        assert _rel(got, base) < 3e-2, (k, _rel(got, base))


@pytest.mark.gpu
def test_deq_fused_adjoint_step(gpu_ext, monkeypatch):
    """The adjoint update fused into the VJP kernel (u_new = J^T u + grad, |u_new - u|^2, the
    device-side convergence flag) against the VJP + adjoint_step pair."""
    from fluxmpi_amd.ops import deq_cell
    cell, z, x = _cell_inputs(seed=2)
    _, state = cell.forward_state(z, x)
    u = torch.randn_like(z)
    g = torch.randn_like(z)
    flag = torch.full((1,), -1.0, device="cuda")
    big = torch.tensor(1e30, device="cuda")
    un_f, ss_f = cell.adjoint_step(state, u, g, big, flag)
    assert float(flag) == 1.0
    monkeypatch.setattr(deq_cell, "ENABLED", False)
    un_u, ss_u = cell.adjoint_step(state, u, g)
    assert _rel(un_f, un_u) < 3e-2
    assert abs(float(ss_f) - float(ss_u)) <= 5e-2 * float(ss_u)
    # the flag is exactly ss <= thresh2
    monkeypatch.setattr(deq_cell, "ENABLED", True)
    _, ss2 = cell.adjoint_step(state, u, g, torch.tensor(float(ss_f) * 0.5, device="cuda"), flag)
    assert float(flag) == 0.0 and float(ss2) == float(ss_f)


def worker_deq_cifar_functional():
    """The FastDEQ-width DEQ's nested (irregular) parameter tree through bench.py's functional
    step — allreduce_gradients(gs, op=AVG, like=ps) then Optimisers.update! — on 2 gloo ranks with
    different data: the ranks end with identical parameters, equal to one process applying the
    mean of both ranks' gradients."""
    import importlib.util
    import os

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models import build_model

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def data(k):
        g = torch.Generator().manual_seed(50 + k)
        return torch.randn(2, 3, 32, 32, generator=g), torch.randint(0, 10, (2,), generator=g)

    def model():
        torch.manual_seed(9)
        return build_model("deq_cifar", ch=32, groups=8, max_iter=6, tol=0.0, bwd_iter=6, bwd_tol=0.0)

    m = model()
    f = bench.Functional(FluxMPI, O, m, O.Descent(0.1))
    assert f.comm_summary()["communicate"] and sum(f.comm_summary()["bucket_mb"]) > 0
    x, y = data(r)
    F.cross_entropy(f(x), y).backward()
    f.step()
    # reference: one process, mean of both ranks' gradients
    ref = model()
    grads = []
    for k in range(W):
        ref.zero_grad()
        xk, yk = data(k)
        F.cross_entropy(ref(xk), yk).backward()
        grads.append([p.grad.clone() for p in ref.parameters()])
    with torch.no_grad():
        for i, p in enumerate(ref.parameters()):
            p -= 0.1 * sum(g[i] for g in grads) / W
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-4, atol=1e-5, msg=n)
        g = FluxMPI.allgather(p.detach().clone())
        assert torch.equal(g[0], g[1]), n
    FluxMPI.Finalize()


def test_deq_cifar_functional_gloo(spmd):
    spmd("tests.test_deq:worker_deq_cifar_functional", timeout=300)


def worker_functional_bf16_masters():
    """bench.py's functional step on bf16 parameters: Optimisers.update! runs on fp32 copies (a
    BFloat16 beta2 rounds to 1 and would make Adam 0/0) and the bf16 parameters are refreshed
    from them; both ranks end identical and equal to fp32 Adam on the averaged bf16 gradients."""
    import importlib.util
    import os

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def model():
        torch.manual_seed(4)
        return torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3)).bfloat16()

    def data(k):
        g = torch.Generator().manual_seed(70 + k)
        return torch.randn(4, 6, generator=g).bfloat16()

    m = model()
    f = bench.Functional(FluxMPI, O, m, O.Adam(1e-2))
    assert len(f.low) == 4  # every bf16 leaf has an fp32 copy
    for _ in range(2):
        m(data(r)).float().pow(2).mean().backward()
        f.step()
    # reference: fp32 masters, Adam on the mean of both ranks' bf16 gradients
    ref = model()
    ps = {n: p.detach().float().clone() for n, p in ref.named_parameters()}
    st = O.setup(O.Adam(1e-2), ps)
    for _ in range(2):
        gs = {}
        for k in range(W):
            ref.zero_grad()
            ref(data(k)).float().pow(2).mean().backward()
            for n, p in ref.named_parameters():
                gs[n] = gs.get(n, 0) + p.grad.float() / W
        gs = {n: g.bfloat16() for n, g in gs.items()}  # the bf16 gradient the allreduce delivers
        st, ps = O.update(st, ps, gs)
        with torch.no_grad():
            for n, p in ref.named_parameters():
                p.copy_(ps[n])
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        assert p.dtype == torch.bfloat16 and torch.isfinite(p.float()).all(), n
        torch.testing.assert_close(p.float(), q.float(), rtol=2e-2, atol=2e-2, msg=n)
        g = FluxMPI.allgather(p.detach().float().clone())
        assert torch.equal(g[0], g[1]), n
    FluxMPI.Finalize()


def test_functional_bf16_masters_gloo(spmd):
    spmd("tests.test_deq:worker_functional_bf16_masters", timeout=300)


def test_skip_deq_initial_guess_and_aux_gradient_cpu():
    """Skip DEQ (FastDEQ.jl's explicit initial-guess network): the solve starts at skip(x), the
    skip convolution is trained by the auxiliary loss only, and the classifier's loss gradient is
    unchanged by it (same fixed point up to the solver tolerance)."""
    torch.manual_seed(0)
    m = deq_mnist(tol=1e-5, max_iter=60, bwd_tol=1e-5, bwd_iter=60, skip=1, skip_reg=1.0)
    assert m.deq.skip is not None and m.deq.skip.weight.shape == (48, 48, 3, 3)
    assert float(m.deq.skip.weight.detach().abs().sum()) == 0.0  # zero init: the first solve starts at 0
    x = torch.randn(2, 1, 28, 28)
    y = torch.randint(0, 10, (2,))
    F.cross_entropy(m(x), y).backward()
    g = m.deq.skip.weight.grad
    assert g is not None and torch.isfinite(g).all() and float(g.abs().sum()) > 0
    assert m.deq.last_skip_res is not None and abs(float(m.deq.last_skip_res) - 1.0) < 1e-4  # 0 vs z*
    # a trained-looking guess: the fixed point and the head gradient do not depend on it
    m2 = deq_mnist(tol=1e-5, max_iter=60, bwd_tol=1e-5, bwd_iter=60)
    m2.load_state_dict({k: v for k, v in m.state_dict().items() if not k.startswith("deq.skip")})
    with torch.no_grad():
        m.deq.skip.weight.normal_(0, 0.05)
    m.zero_grad()
    m2.zero_grad()
    F.cross_entropy(m(x), y).backward()
    F.cross_entropy(m2(x), y).backward()
    torch.testing.assert_close(m.head.weight.grad, m2.head.weight.grad, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("bwd_m", [3, 5])
def test_anderson_adjoint_matches_fixed_point_adjoint_cpu(bwd_m):
    """The adjoint solve by Anderson(bwd_m) (per-sample normalised right-hand side) gives the
    parameter gradients of a tightly converged fixed-point adjoint, in a fraction of its
    iterations (its residual test is relative to h(u) = J^T u + g, the forward's kind of test)."""
    torch.manual_seed(0)
    x = torch.randn(3, 1, 28, 28)
    y = torch.randint(0, 10, (3,))
    grads, iters = [], []
    for m_, tol in ((0, 1e-6), (bwd_m, 1e-3)):
        torch.manual_seed(1)
        m = deq_mnist(tol=1e-6, max_iter=60, bwd_tol=tol, bwd_iter=200, bwd_m=m_)
        F.cross_entropy(m(x), y).backward()
        grads.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
        iters.append(m.deq.last_bwd_iters)
    ref, got = grads
    assert ref.keys() == got.keys()
    err = sum((got[k] - ref[k]).square().sum() for k in ref).sqrt() / sum(ref[k].square().sum() for k in ref).sqrt()
    assert float(err) < 5e-3, float(err)
    assert iters[1] * 3 < iters[0], iters


def test_anderson_restart_same_fixed_point_cpu():
    """anderson(restart=r): a history restart from the newest iterate on a stall keeps the fixed
    point and the iteration accounting (every segment's evaluations count against max_iter)."""
    torch.manual_seed(0)
    d = 64
    A = torch.randn(4, d, d) / d ** 0.5
    A = 0.97 * A / torch.linalg.matrix_norm(A, ord=2).view(-1, 1, 1)  # slowly contracting
    b = torch.randn(4, d)
    calls = []

    def f(z):
        calls.append(1)
        return torch.einsum("bij,bj->bi", A, z) + b

    ref = torch.linalg.solve(torch.eye(d) - A, b)
    for r in (0, 1, 2):
        calls.clear()
        z, it, res = anderson(f, torch.zeros(4, d), m=3, max_iter=200, tol=1e-6, restart=r)
        torch.testing.assert_close(z, ref, rtol=1e-4, atol=1e-4)
        assert it <= 200 and len(calls) == it + 1, (r, it, len(calls))
    # a map without a fixed point (residual ~ 1 / k): the stall test fires, the restarted solve
    # takes a different path, and the evaluations still match the reported count
    outs = []
    for r in (0, 1):
        calls.clear()
        z, it, res = anderson(lambda v: (calls.append(1), v + 1.0)[1], torch.zeros(2, 16), m=3, max_iter=40,
                              tol=0.0, restart=r)
        assert it == 39 and len(calls) == 40, (r, it, len(calls))
        outs.append(float(res))
    assert outs[0] != outs[1], outs
