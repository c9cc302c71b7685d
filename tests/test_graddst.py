"""Direct gradient delivery (ops/graddst.py): weight gradients born in the DDP bucket slices.

CPU/gloo: a Linear whose backward allocates its weight gradient with ``graddst.empty`` (as the
package's HIP weight-gradient ops do) under a 2-rank DDP in "steal" mode. The applied update
must equal the summed-gradient reference, the gradients must lie in the bucket (no pack copy),
and the corner cases fall back to fresh tensors: a weight used twice in one graph, gradient
accumulation under ``no_sync``, ``step(zero_grad=False)``.
"""
import torch

from fluxmpi_amd.ops import graddst


class _DLin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        with graddst.into(w):
            gw = graddst.empty(tuple(w.shape), w.dtype, w.device)
        torch.matmul(dy.t(), x, out=gw)
        return dy @ w, gw


class _Net(torch.nn.Module):
    def __init__(self, seed, shared=False):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w1 = torch.nn.Parameter(torch.randn(16, 5, generator=g) * 0.3)
        self.w2 = torch.nn.Parameter(torch.randn(16, 16, generator=g) * 0.3)
        self.w3 = torch.nn.Parameter(torch.randn(1, 16, generator=g) * 0.3)
        self.shared = shared

    def forward(self, x):
        h = torch.tanh(_DLin.apply(x, self.w1))
        h = torch.tanh(_DLin.apply(h, self.w2))
        if self.shared:  # w2 twice: autograd sums its two gradients
            h = torch.tanh(_DLin.apply(h, self.w2))
        return _DLin.apply(h, self.w3)


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(8, 5, generator=g)
    return x, x.sum(1, keepdim=True) ** 2


def test_take_semantics():
    p = torch.nn.Parameter(torch.zeros(4, 3))
    flat = torch.zeros(20)
    assert graddst.take(p, (4, 3), p.dtype) is None  # nothing attached
    graddst.attach(p, flat, 4)
    assert graddst.take(p, (3, 3), p.dtype) is None  # size mismatch
    assert graddst.take(p, (12,), torch.float64) is None  # dtype mismatch
    t = graddst.take(p, (12,), p.dtype)
    assert t is not None and t.data_ptr() == flat.data_ptr() + 4 * 4
    assert graddst.take(p, (12,), p.dtype) is None  # once per backward
    graddst.rearm(p)
    p.grad = torch.ones(4, 3)
    assert graddst.take(p, (12,), p.dtype) is None  # a gradient is already there
    p.grad = None
    with graddst.into(p):
        a = graddst.empty((4, 3), p.dtype, "cpu")
        b = graddst.empty((4, 3), p.dtype, "cpu")  # the binding is used up
    assert a.data_ptr() == flat.data_ptr() + 16 and b.data_ptr() != a.data_ptr()
    graddst.detach(p)
    graddst.rearm(p)
    assert graddst.take(p, (12,), p.dtype) is None


def test_empty_like_channels_last_filter():
    """A channels_last filter's gradient lands in its bucket slice with the filter's strides (the
    stem / 3x3 weight-gradient kernels write it in that layout)."""
    p = torch.nn.Parameter(torch.zeros(8, 3, 7, 7).contiguous(memory_format=torch.channels_last))
    flat = torch.zeros(p.numel() + 10)
    graddst.attach(p, flat, 10)
    g = graddst.empty_like(p)
    assert g.shape == p.shape and g.stride() == p.stride() and g.data_ptr() == flat.data_ptr() + 40
    graddst.detach(p)
    graddst.rearm(p)
    assert graddst.empty_like(p).stride() == p.stride()  # not attached: a fresh tensor, same layout
    assert not graddst._dense(torch.zeros(4, 6)[:, :3])


def _reference(shared, W, steps, lr):
    ref = _Net(1000, shared)
    for _ in range(steps):
        ref.zero_grad()
        for k in range(W):
            xk, yk = _data(k)
            ((ref(xk) - yk) ** 2).mean().backward()
        with torch.no_grad():
            for p in ref.parameters():
                p -= lr * p.grad
    return ref


def worker_graddst():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    for shared in (False, True):
        model = _Net(1000 + r, shared)
        ddp = DDP(model, O.Descent(0.1), bucket_mb=0.0008, first_bucket_mb=0.0004, grad_mode="steal")
        assert ddp.direct_grads and len(ddp.buckets) > 1
        x, y = _data(r)
        for _ in range(3):
            before = ddp.pack_copies
            ((ddp(x) - y) ** 2).mean().backward()
            ddp.step()
            # born in the bucket (no pack copy): all but w2 when it is used twice (autograd sums
            # its two gradients into a fresh tensor, which the pack copies)
            assert ddp.pack_copies - before == (1 if shared else 0)
        ref = _reference(shared, W, 3, 0.1)
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-5)
        # gradient accumulation: two half batches under no_sync == one full batch
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
        ddp.zero_grad()
    # step(zero_grad=False): applied S1 + S2, direct delivery on both backwards
    model = _Net(1000 + r)
    ddp = DDP(model, O.Descent(0.1), grad_mode="steal")
    x, y = _data(r)
    ((ddp(x) - y) ** 2).mean().backward()
    ddp.step(zero_grad=False)
    ((ddp(x) - y) ** 2).mean().backward()
    ddp.step()
    ref = _Net(1000)
    grads = []
    for _ in range(2):
        ref.zero_grad()
        for k in range(W):
            xk, yk = _data(k)
            ((ref(xk) - yk) ** 2).mean().backward()
        grads.append([p.grad.clone() for p in ref.parameters()])
        with torch.no_grad():
            for p, g0 in zip(ref.parameters(), grads[0]):
                p -= 0.1 * (g0 if len(grads) == 1 else p.grad + g0)
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-5)
    FluxMPI.Finalize()


def test_graddst_gloo(spmd):
    spmd("tests.test_graddst:worker_graddst", timeout=120)


def test_no_attachment_without_communication():
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    model = _Net(3)
    ddp = DDP(model, O.Descent(0.1))  # world of one, not forced: nothing to reduce, no buckets used
    assert not ddp.direct_grads
    x, y = _data(0)
    ((ddp(x) - y) ** 2).mean().backward()
    assert not any(graddst.delivered(p) for p in model.parameters())
    ddp.step()
    assert ddp.pack_copies == 0
