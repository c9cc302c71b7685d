"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = [torch.float32, torch.bfloat16, torch.float16]


def _tensors(dtype, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(1,), (7,), (8,), (9,), (33, 3), (1000,), (4097,), (8192,), (8193,), (3, 224, 5), (64, 64, 3, 3)]
    out = [torch.randn(s, generator=g).to(dtype).to(dev) for s in shapes]
    # an unaligned view (storage offset 1) exercises the scalar path
    base = torch.randn(1001, generator=g).to(dtype).to(dev)
    out.append(base[1:])
    return out


@pytest.mark.parametrize("src_dt", DT)
@pytest.mark.parametrize("dst_dt", DT)
def test_pack_unpack(gpu_ext, src_dt, dst_dt):
    from fluxmpi_amd.ops import multi_tensor as mt
    dev = torch.device("cuda")
    ts = _tensors(src_dt, dev)
    offs, total = mt.aligned_offsets([t.numel() for t in ts], dst_dt)
    flat = torch.full((total,), float("nan"), dtype=dst_dt, device=dev)
    mt.pack(ts, flat, offs, scale=0.5)
    for t, o in zip(ts, offs):
        ref = (t.float() * 0.5).to(dst_dt).reshape(-1)
        assert torch.equal(flat[o:o + t.numel()], ref)
    outs = [torch.empty_like(t) for t in ts]
    mt.unpack(flat, outs, offs, scale=2.0)
    for t, o, u in zip(ts, offs, outs):
        ref = (flat[o:o + t.numel()].float() * 2.0).to(src_dt).reshape(t.shape)
        assert torch.equal(u, ref)


def test_many_tensors_and_large(gpu_ext):
    """>40 tensors (several launches) and a multi-chunk tensor."""
    from fluxmpi_amd.ops import multi_tensor as mt
    dev = torch.device("cuda")
    ts = [torch.randn(i * 37 + 1, device=dev) for i in range(130)] + [torch.randn(3_000_001, device=dev)]
    offs, total = mt.aligned_offsets([t.numel() for t in ts], torch.float32)
    flat = torch.zeros(total, device=dev)
    mt.pack(ts, flat, offs)
    ref = torch.cat([t for t in ts])
    got = torch.cat([flat[o:o + t.numel()] for t, o in zip(ts, offs)])
    assert torch.equal(got, ref)


def test_scale_fill_sumsq(gpu_ext):
    from fluxmpi_amd.ops import multi_tensor as mt
    dev = torch.device("cuda")
    ts = _tensors(torch.float32, dev, 1)
    ref = [t * 3.0 for t in ts]
    mt.scale_(ts, 3.0)
    for t, r in zip(ts, ref):
        assert torch.equal(t, r)
    s = mt.sumsq(ts)
    exp = sum(float((t.double() ** 2).sum()) for t in ts)
    assert abs(float(s) - exp) / exp < 1e-5
    mt.fill_(ts, 0.25)
    assert all(torch.all(t == 0.25) for t in ts)
    bf = _tensors(torch.bfloat16, dev, 2)
    mt.fill_(bf, -1.0)
    assert all(torch.all(t == -1) for t in bf)


COMBOS = [
    (torch.float32, torch.float32, torch.float32, False),
    (torch.float32, torch.bfloat16, torch.float32, False),  # fp32 parameters, bf16 gradients
    (torch.bfloat16, torch.bfloat16, torch.bfloat16, False),
    (torch.bfloat16, torch.bfloat16, torch.float32, True),
    (torch.bfloat16, torch.float32, torch.float32, True),
    (torch.float16, torch.float16, torch.float32, True),
]


@pytest.mark.parametrize("pd,gd,sd,master", COMBOS)
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adam(gpu_ext, pd, gd, sd, master, wd):
    from fluxmpi_amd.ops import optim
    dev = torch.device("cuda")
    g0 = torch.Generator().manual_seed(3)
    shapes = [(5,), (8,), (4096,), (4099,), (300, 7), (10000,)]
    P = [torch.randn(s, generator=g0) for s in shapes]
    G = [torch.randn(s, generator=g0) for s in shapes]
    M = [torch.randn(s, generator=g0) * 0.1 for s in shapes]
    V = [torch.rand(s, generator=g0) * 0.1 for s in shapes]

    def mk(lst, dt):
        return [t.to(dt).to(dev) for t in lst]

    p1, g1, m1, v1 = mk(P, pd), mk(G, gd), mk(M, sd), mk(V, sd)
    w1 = mk(P, torch.float32) if master else None
    p2, g2, m2, v2 = [t.clone() for t in p1], [t.clone() for t in g1], [t.clone() for t in m1], [t.clone() for t in v1]
    w2 = [t.clone() for t in w1] if master else None
    kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, bc1=1 - 0.9 ** 3, bc2=1 - 0.999 ** 3, weight_decay=wd,
              grad_scale=0.5)
    for _ in range(2):
        optim.adam_(p1, g1, m1, v1, masters=w1, **kw)
        # oracle: same math on CPU in fp32
        pc, gc, mc, vc = [t.cpu() for t in p2], [t.cpu() for t in g2], [t.cpu() for t in m2], [t.cpu() for t in v2]
        wc = [t.cpu() for t in w2] if master else None
        optim.adam_reference_(pc, gc, mc, vc, masters=wc, **kw)
        for dst, src in zip(p2 + m2 + v2 + (w2 or []), pc + mc + vc + (wc or [])):
            dst.copy_(src)
    tol = dict(rtol=1e-6, atol=1e-7) if pd == torch.float32 else dict(rtol=1e-2, atol=1e-3)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a.float(), b.float(), **tol)
    stol = dict(rtol=1e-6, atol=1e-7) if sd == torch.float32 else dict(rtol=1e-2, atol=1e-3)
    for a, b in zip(m1 + v1, m2 + v2):
        torch.testing.assert_close(a.float(), b.float(), **stol)
    if master:
        for a, b in zip(w1, w2):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_adam_device_hyper(gpu_ext):
    """Graph-mode scalars (lr, beta^t on device) give the same result as host scalars."""
    from fluxmpi_amd.ops import optim
    dev = torch.device("cuda")
    p = torch.randn(10000, device=dev)
    g = torch.randn(10000, device=dev)
    m = torch.zeros_like(p); v = torch.zeros_like(p)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    hyper = torch.tensor([1e-3, 0.9, 0.999], device=dev)
    for t in range(1, 4):
        optim.adam_([p], [g], [m], [v], lr=0, beta1=0.9, beta2=0.999, eps=1e-8, bc1=0, bc2=0, dev_hyper=hyper)
        optim.adam_advance_(hyper, 0.9, 0.999)
        optim.adam_([p2], [g], [m2], [v2], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                    bc1=1 - float(torch.tensor(0.9) ** t), bc2=1 - float(torch.tensor(0.999) ** t))
    torch.testing.assert_close(p, p2, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("mom,nest", [(0.0, False), (0.9, False), (0.9, True)])
def test_fused_sgd(gpu_ext, mom, nest):
    from fluxmpi_amd.ops import optim
    dev = torch.device("cuda")
    P = [torch.randn(s, device=dev) for s in [(3,), (4096,), (5000,)]]
    G = [torch.randn_like(t) for t in P]
    B = [torch.randn_like(t) for t in P]
    P2, B2 = [t.cpu() for t in P], [t.cpu() for t in B]
    optim.sgd_(P, G, B, lr=0.1, momentum=mom, nesterov=nest, weight_decay=0.01)
    optim.sgd_reference_(P2, [g.cpu() for g in G], B2, lr=0.1, momentum=mom, nesterov=nest, weight_decay=0.01)
    for a, b in zip(P + B, P2 + B2):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-6, atol=1e-6)


def test_rccl_world1(gpu_ext):
    """The native RCCL communicator initialises and runs collectives on one GPU."""
    from fluxmpi_amd.parallel.comm import RcclComm
    c = RcclComm(0, 1, torch.device("cuda", 0))
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    ref = x.clone()
    c.allreduce(x)
    c.broadcast(x, 0)
    w = c.allreduce(x, "max", async_op=True)
    w.wait()
    y = torch.empty_like(x)
    c.allreduce_out(x, y)
    c.allreduce_coalesced([x, y])
    torch.cuda.synchronize()
    assert torch.equal(x, ref) and torch.equal(y, ref)
    assert c.version >= 22000
    c.check_async_error()
    c.destroy()


def test_optimisers_update_gpu_matches_cpu(gpu_ext):
    """Functional Optimisers.update on GPU (fused path) == CPU path (reference math)."""
    from fluxmpi_amd import optimisers as O
    ps = {"w": torch.randn(300, 7), "b": torch.randn(7)}
    gs = {"w": torch.randn(300, 7), "b": torch.randn(7)}
    st = O.setup(O.Adam(1e-2), ps)
    psg = {k: v.cuda() for k, v in ps.items()}
    gsg = {k: v.cuda() for k, v in gs.items()}
    stg = O.setup(O.Adam(1e-2), psg)
    for _ in range(3):
        st, ps = O.update(st, ps, gs)
        stg, psg = O.update(stg, psg, gsg)
    for k in ps:
        torch.testing.assert_close(psg[k].cpu(), ps[k], rtol=1e-5, atol=1e-6)
    assert stg["w"].state[2] == st["w"].state[2]


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 7, 16, 17, 100, 788, 2048, 2049, 5000])
@pytest.mark.parametrize("n", [1, 4, 768, 1000, 3072, 6])
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_splitk_reduce(gpu_ext, S, n, odt):
    """gemm_splitk_reduce over S partial rows (one launch, the column-reduction kernel for
    16 < S <= 2048 and n % 4 == 0; the G-ary tree otherwise) vs torch.sum in fp64."""
    from fluxmpi_amd.ops import _ext
    from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE
    torch.manual_seed(S + n)
    ws = torch.randn(S, n, device="cuda")
    want = ws.double().sum(0)
    out = torch.empty(n, device="cuda", dtype=odt)
    scratch = ws.clone()  # the tree path reduces in place
    _ext.get(required=True).gemm_splitk_reduce(scratch.data_ptr(), S, n, out.data_ptr(), DTYPE_CODE[odt],
                                               torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    tol = 1e-4 * S ** 0.5 if odt == torch.float32 else 1e-2 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(out.double(), want.to(odt).double() if odt != torch.float32 else want,
                               rtol=1e-3 if odt == torch.float32 else 1e-2, atol=tol)
