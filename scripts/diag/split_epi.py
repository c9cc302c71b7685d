"""Debug: gemm_nt split tail vs unsplit per epilogue; prints where outputs differ (tile rows / cols)."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import _ext

C = _ext.get(required=True)
st = torch.cuda.current_stream().cuda_stream


def uni(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def run(m, n, k, epi, sm):
    torch.manual_seed(0)
    a = uni(m, k)
    w = (uni(n, k) * k ** -0.5).bfloat16()
    bias = (torch.rand(n, device="cuda") - 0.5).float()
    c = torch.zeros(m, n, device="cuda", dtype=torch.bfloat16)
    c2 = torch.zeros_like(c)
    h = uni(m, n)
    part = torch.zeros(C.gemm_nt_colpart_rows(m), n, device="cuda")
    C.gemm_nt_set_split(sm)
    C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), c2.data_ptr() if epi == 1 else 0,
              bias.data_ptr() if epi in (0, 1) else 0, 1, h.data_ptr() if epi == 2 else 0,
              part.data_ptr() if epi == 2 else 0, k, k, n, m, n, k, epi, st)
    torch.cuda.synchronize()
    return c.float(), c2.float(), part


for (m, n, k) in [(256, 256, 8192), (50432, 768, 2304)]:
    for epi in (0, 1, 2):
        c0, g0, p0 = run(m, n, k, epi, 0)
        c1, g1, p1 = run(m, n, k, epi, 8)
        for nm, x0, x1 in (("c", c0, c1), ("c2", g0, g1), ("part", p0, p1)):
            d = (x1 - x0).abs()
            rel = float(d.max() / x0.abs().max().clamp_min(1e-9))
            bad = (d > 0.05 * x0.abs().max()).nonzero()
            info = ""
            if len(bad):
                r, cc = bad[:, 0], bad[:, 1]
                info = (f" nbad={len(bad)} rows%256 {sorted(set((r % 256 // 16).tolist()))[:16]} "
                        f"cols%256 {sorted(set((cc % 256 // 16).tolist()))[:16]} tiles_m {sorted(set((r // 256).tolist()))[:8]} "
                        f"nan={int(torch.isnan(x1).sum())}")
            print(f"m{m} n{n} k{k} epi{epi} {nm}: rel {rel:.3g}{info}", flush=True)
