"""Where does gemm_nt EPI 1's derivative output go wrong? (NaN / error pattern by tile position)"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 1)[0] + "/diag")
import load_variant  # noqa: E402  (FLUXMPI_C_VARIANT=<.so>: e.g. gemm_nt.hip built with SLP vectorisation)

load_variant.install()
from fluxmpi_amd.ops import gelu as GL  # noqa: E402
from fluxmpi_amd.ops import gemm_nt as G  # noqa: E402

print("library:", sys.modules["fluxmpi_amd._C"].__file__ if "fluxmpi_amd._C" in sys.modules else "package default")
for form, m, n, k in (("tanh", 512, 512, 128), ("tanh", 50432, 2304, 768), ("tanh", 50432, 3072, 768),
                      ("erf", 50432, 3072, 768)):
    GL.set_form(form)
    print("form", form)
    torch.manual_seed(0)
    x = ((torch.rand(m, k, device="cuda") * 2 - 1)).bfloat16()
    w = ((torch.rand(n, k, device="cuda") * 2 - 1) * k ** -0.5).bfloat16()
    b = (torch.randn(n, device="cuda") * 0.5).float()
    y = G.linear_fwd(x, w, b)
    d = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
    g = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
    d2, g2 = G.linear_fwd(x, w, b, gelu=True)
    torch.cuda.synchronize()
    ref_d = GL._gelu_grad_ref(y.float())
    ref_g = GL.gelu(y.float())
    for name, got, ref in (("d", d2, ref_d), ("g", g2, ref_g)):
        bad = ~torch.isfinite(got.float())
        err = (got.float() - ref).abs()
        err[bad] = float("inf")
        big = err > 0.05
        idx = big.nonzero()
        print(name, m, n, "nonfinite", int(bad.sum()), "big", int(big.sum()), "max err", float(err[~bad].max()) if (~bad).any() else None)
        if idx.numel():
            r, c = idx[:, 0], idx[:, 1]
            print("  rows%256 uniq", sorted(set((r % 256).tolist()))[:40])
            print("  cols%256 uniq", sorted(set((c % 256).tolist()))[:40])
            print("  first", [(int(a), int(bb), float(got[a, bb]), float(ref[a, bb]), float(y[a, bb])) for a, bb in idx[:8].tolist()])
