"""gemm_nt.hip (ViT forward / input-gradient GEMMs with fused epilogues) vs PyTorch fp32: every
ViT-B/16 Linear shape at batch 256 (M = 50432 tokens), plus odd k-tile counts, the minimum K and
tile counts that are not a multiple of the CU count (the persistent kernel's tile stream and its
LDS buffer parity cross tile boundaries), fewer tiles than CUs, and the implicit-GEMM 3x3
convolution / BatchNorm-statistics epilogues."""
import pytest
import torch

pytestmark = pytest.mark.gpu

M_VIT = 50432
# (name, rows, N, K): forward x W^T and input gradient dy W of qkv / proj / fc1 / fc2
VIT_FWD = [("qkv", M_VIT, 2304, 768), ("proj", M_VIT, 768, 768), ("fc1", M_VIT, 3072, 768),
           ("fc2", M_VIT, 768, 3072)]
VIT_DGRAD = [("qkv", M_VIT, 2304, 768), ("proj", M_VIT, 768, 768), ("fc1", M_VIT, 3072, 768),
             ("fc2", M_VIT, 768, 3072)]  # (rows, N_out, N_in): dx [rows, N_in] = dy [rows, N_out] W
SMALL = [(512, 768, 768), (768, 256, 3072), (256 * 41, 768, 832), (256 * 37, 512, 128), (256 * 300, 256, 192)]
# one tile with a long K, a few tiles (fewer than CUs), one tile per workgroup
FEW_TILES = [(256, 256, 8192), (512, 768, 4096), (256, 512, 1344), (1024, 1024, 2048)]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.fixture(params=["tanh", "erf"])
def gelu_form(request):
    from fluxmpi_amd.ops import gelu as GL
    old = GL.FORM
    GL.set_form(request.param)
    yield request.param
    GL.set_form(old)


def _uni(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).bfloat16()


def _check_fwd(m, n, k, bias, gelu_form=None):
    from fluxmpi_amd.ops import gelu as GL
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(0)
    x = _uni(m, k)
    w = _uni(n, k, scale=k ** -0.5)
    b = None if bias is None else (torch.randn(n, device="cuda") * 0.5).to(torch.float32 if bias == "f32" else torch.bfloat16)
    assert G.supported(m, n, k, x, w, fused=True)
    y = G.linear_fwd(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    assert _rel(y, ref) < 5e-3
    if gelu_form is not None:
        d, g = G.linear_fwd(x, w, b, gelu=True)
        assert _rel(g, GL.gelu(y.float())) < 5e-3  # GELU of the rounded pre-activation
        assert _rel(d, GL._gelu_grad_ref(y.float())) < 5e-3  # and its derivative


def _check_dgrad(m, n_out, n_in, gelu_form=None):
    from fluxmpi_amd.ops import gelu as GL
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(1)
    dy = _uni(m, n_out)
    w = _uni(n_out, n_in, scale=n_out ** -0.5)
    assert G.supported(m, n_in, n_out, dy, w, fused=True)
    dx = G.linear_dgrad(dy, w)
    ref = dy.float() @ w.float()
    assert _rel(dx, ref) < 5e-3
    if gelu_form is not None:
        h = _uni(m, n_in, scale=3.0)
        d = GL._gelu_grad_ref(h.float()).bfloat16()  # the derivative as EPI 1 stores it
        dh, db = G.linear_dgrad(dy, w, gelu_d=d)
        dh_ref = ref.bfloat16().float() * GL._gelu_grad_ref(h.float())
        assert _rel(dh, dh_ref) < 5e-3
        torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-3, atol=2e-2)
        _, db16 = G.linear_dgrad(dy, w, gelu_d=d, bias_dtype=torch.bfloat16)
        assert db16.dtype == torch.bfloat16 and _rel(db16, db) < 1e-2


@pytest.mark.parametrize("name,m,n,k", VIT_FWD)
@pytest.mark.parametrize("bias", [None, "f32", "bf16"])
def test_vit_fwd(gpu_ext, name, m, n, k, bias):
    _check_fwd(m, n, k, bias)


@pytest.mark.parametrize("name,m,n,k", VIT_FWD)
def test_vit_fwd_gelu(gpu_ext, gelu_form, name, m, n, k):
    _check_fwd(m, n, k, "f32", gelu_form)


@pytest.mark.parametrize("name,m,n_out,n_in", VIT_DGRAD)
def test_vit_dgrad(gpu_ext, gelu_form, name, m, n_out, n_in):
    _check_dgrad(m, n_out, n_in, gelu_form)


@pytest.mark.parametrize("m,n,k", SMALL)
def test_small_and_odd_shapes(gpu_ext, gelu_form, m, n, k):
    _check_fwd(m, n, k, "bf16", gelu_form)
    if k % 256 == 0:  # dgrad: dx [m, k] = dy [m, n] W [n, k]: k is the output width
        _check_dgrad(m, n, k, gelu_form)


@pytest.mark.parametrize("m,n,k", FEW_TILES)
def test_few_tiles_long_k(gpu_ext, m, n, k):
    for _ in range(2):
        _check_fwd(m, n, k, "f32", "tanh")
    if k % 256 == 0:
        _check_dgrad(m, n, k, "tanh")


def test_transpose_bf16(gpu_ext):
    from fluxmpi_amd.ops import gemm_nt as G
    for r, c in ((768, 3072), (3072, 768), (40, 72), (2304, 768)):
        w = torch.randn(r, c, device="cuda").bfloat16()
        assert torch.equal(G.weight_t(w), w.t())


def test_unsupported_shapes(gpu_ext):
    from fluxmpi_amd.ops import gemm_nt as G
    x = torch.zeros(200, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(768, 768, device="cuda", dtype=torch.bfloat16)
    assert not G.supported(200, 768, 768, x, w, fused=True)  # rows not a multiple of 256
    assert not G.supported(256, 768, 768, x.float(), w, fused=True)
    assert not G.supported(256, 768, 64, x, w, fused=True)  # K < 128
    assert not G.supported(256, 768, 96, x, w, fused=True)  # K not a multiple of 64


# (nimg, H, W, C, Cout): output pixels tile by 256; odd image sizes (rows of a tile span images,
# every padding case), the ResNet-50 stage-3/4 widths
CONV_SHAPES = [(4, 8, 8, 64, 256), (256, 5, 7, 128, 256), (64, 14, 14, 256, 256), (256, 7, 7, 512, 512)]


@pytest.fixture
def any_shape(monkeypatch):
    """The kernel on every shape it supports (the routing's tile-count / K thresholds off)."""
    from fluxmpi_amd.ops import gemm_nt as G
    monkeypatch.setattr(G, "MIN_TILES", 0)
    monkeypatch.setattr(G, "MIN_K", 0)
    monkeypatch.setattr(G, "CONV", True)


@pytest.mark.parametrize("nimg,h,w,c,co", CONV_SHAPES)
def test_conv3x3_fwd_stats_and_dgrad(gpu_ext, any_shape, nimg, h, w, c, co):
    import torch.nn.functional as F
    from fluxmpi_amd.ops import gemm as GM
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(2)
    x = _uni(nimg, c, h, w).contiguous(memory_format=torch.channels_last)
    wt = _uni(co, c, 3, 3, scale=(9 * c) ** -0.5).contiguous(memory_format=torch.channels_last)
    M = nimg * h * w
    assert G.conv_ok(M, c, co, x)
    stats = torch.zeros(GM.SHARDS, 2, co, device="cuda")
    for _ in range(2):
        stats.zero_()
        y = GM.conv3x3_fwd(x, wt, stats=stats)
        ref = F.conv2d(x.float(), wt.float(), padding=1)
        assert _rel(y, ref) < 5e-3
    yf = y.float().permute(0, 2, 3, 1).reshape(M, co)
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    if G.conv_ok(M, co, c, x):  # input gradient: the same kernel on the flipped transpose
        dy = _uni(nimg, co, h, w).contiguous(memory_format=torch.channels_last)
        GM.note_filter(wt)
        dx = GM.conv3x3_dgrad(dy, wt)
        dref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), padding=1)
        assert _rel(dx, dref) < 5e-3
        # + a residual summand in the epilogue (EPI 4): exactly bf16(bf16(conv) + r)
        res = _uni(nimg, c, h, w).contiguous(memory_format=torch.channels_last)
        dxr = GM.conv3x3_dgrad(dy, wt, residual=res)
        torch.testing.assert_close(dxr, (dx.float() + res.float()).bfloat16(), rtol=0, atol=0)
        assert _rel(dxr, dref + res.float()) < 5e-3


@pytest.mark.parametrize("m,n,k", [(50176, 1024, 256), (12544, 512, 2048), (802816 // 4, 256, 64 * 2)])
def test_conv1x1_stats(gpu_ext, any_shape, m, n, k):
    from fluxmpi_amd.ops import gemm as GM
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(3)
    x = _uni(m, k)
    w = _uni(n, k, scale=k ** -0.5)
    assert G.gemm_ok(m, n, k, x, w)
    stats = torch.zeros(GM.SHARDS, 2, n, device="cuda")
    y = GM.conv1x1_fwd(x, w, stats=stats)
    ref = x.float() @ w.float().t()
    assert _rel(y, ref) < 5e-3
    yf = y.float()
    torch.testing.assert_close(stats[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(stats[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


def test_conv_routing_thresholds(gpu_ext):
    """The default routing takes the 256x256 kernel only where it measured faster: >= 160 output
    tiles and K >= 1024 (ResNet-50 stage 3's 3x3 yes; stage 4's 98 tiles and K = 256 1x1s no)."""
    from fluxmpi_amd.ops import gemm_nt as G
    x = torch.zeros(8, device="cuda", dtype=torch.bfloat16)
    assert G.conv_ok(50176, 256, 256, x)          # 14x14x256 3x3: 196 tiles, K = 2304
    assert not G.conv_ok(12544, 512, 512, x)      # 7x7x512: 98 tiles
    assert G.gemm_ok(50176, 256, 1024, x)         # 1x1 1024 -> 256
    assert not G.gemm_ok(50176, 1024, 256, x)     # K = 256


# ---- split-K tail (the last, partial round cut into k-ranges; pieces summed by the last arriver)
SPLIT_SHAPES = [(M_VIT, 768, 3072), (M_VIT, 768, 2304), (256 * 300, 512, 1024), (256 * 37, 256, 4096),
                (256 * 3, 256, 8192)]


@pytest.fixture
def split_mode():
    from fluxmpi_amd.ops import gemm_nt as G
    prev = G.get_split()  # the production default (0 = off) unless FLUXMPI_GEMM_NT_SPLIT says otherwise
    yield G._set_split
    G._set_split(prev)
    assert G.get_split() == prev


@pytest.mark.parametrize("m,n,k", SPLIT_SHAPES)
def test_split_tail_matches_unsplit_and_is_deterministic(gpu_ext, split_mode, m, n, k):
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(3)
    x = _uni(m, k)
    w = _uni(n, k, scale=k ** -0.5)
    b = (torch.randn(n, device="cuda") * 0.5).bfloat16()
    ref = x.float() @ w.float().t() + b.float()
    outs = {}
    for sm in (0, 2, 8, 16):
        split_mode(sm)
        y1 = G.linear_fwd(x, w, b)
        y2 = G.linear_fwd(x, w, b)
        assert torch.equal(y1, y2), f"split {sm}: two launches differ (non-deterministic fix-up)"
        assert _rel(y1, ref) < 5e-3, sm
        outs[sm] = y1
    # only the fp32 summation order differs: a few bf16 roundings flip by one ulp
    for sm in (2, 8, 16):
        d = (outs[sm].float() - outs[0].float()).abs()
        assert float(d.max()) <= 2.0 ** -6 * float(outs[0].float().abs().max()), sm


def test_split_tail_epilogues(gpu_ext, split_mode, gelu_form):
    """EPI 1 (bias + GELU and its derivative), EPI 2 (GELU backward + bias-gradient partials) and
    EPI 3 (BatchNorm statistics of a 3x3 convolution) through split tiles, against the unsplit run."""
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(4)
    res = {}
    for sm in (0, 2):
        split_mode(sm)
        _check_fwd(M_VIT, 768, 3072, "f32", gelu_form)
        _check_dgrad(M_VIT, 3072, 768, gelu_form)
        _check_dgrad(256 * 41, 768, 3072, gelu_form)
        x = _uni(M_VIT, 3072)
        w = _uni(768, 3072, scale=3072 ** -0.5)
        res[sm] = G.linear_fwd(x, w, None, gelu=True)
    for a, b in zip(res[0], res[2]):
        assert _rel(a, b) < 1e-2


def test_split_tail_conv_stats(gpu_ext, split_mode, any_shape):
    from fluxmpi_amd.ops import gemm_nt as G
    torch.manual_seed(5)
    nimg, h, w_, c, co = 64, 14, 14, 256, 256  # 196 output tiles: every CU shares the tail
    x = _uni(nimg, c, h, w_).contiguous(memory_format=torch.channels_last)
    wt = _uni(co, c, 3, 3, scale=(9 * c) ** -0.5)
    ref = torch.nn.functional.conv2d(x.float(), wt.float(), padding=1).permute(0, 2, 3, 1).reshape(-1, co)
    taps = wt.permute(0, 2, 3, 1).reshape(co, 9 * c).contiguous()
    for sm in (0, 8, 2):
        split_mode(sm)
        y = torch.empty(nimg * h * w_, co, device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(64, 2, co, device="cuda")
        G.conv3x3(x, taps, y, st)
        assert _rel(y, ref) < 5e-3, sm
        s = st.sum(0)
        torch.testing.assert_close(s[0], y.float().sum(0), rtol=2e-3, atol=0.5)
        torch.testing.assert_close(s[1], (y.float() ** 2).sum(0), rtol=2e-3, atol=0.5)
