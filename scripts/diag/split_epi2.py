"""Debug: repeat gemm_nt split launches; for wrong elements print c, the derivative D and c / D vs the
true accumulator, to tell a wrong accumulator (partial sum) from a wrong epilogue input."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 1)[0])
import load_variant  # noqa: E402
load_variant.install()
from fluxmpi_amd.ops import _ext

C = _ext.get(required=True)
st = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
m, n, k = 50432, 768, 2304
a = ((torch.rand(m, k, device="cuda") * 2 - 1)).bfloat16()
w = ((torch.rand(n, k, device="cuda") * 2 - 1) * k ** -0.5).bfloat16()
h = ((torch.rand(m, n, device="cuda") * 2 - 1)).bfloat16()
ref = (a.float() @ w.float().t())
part = torch.zeros(C.gemm_nt_colpart_rows(m), n, device="cuda")
import os
SMS = [int(x) for x in os.environ.get('SMS', '0,8').split(',')]
for epi in (2, 2):
    for sm in SMS:
        C.gemm_nt_set_split(sm)
        nbad_tot = 0
        for it in range(10):
            c = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
            C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), 0, 0, 0, h.data_ptr() if epi == 2 else 0,
                      part.data_ptr() if epi == 2 else 0, k, k, n, m, n, k, epi, st)
            torch.cuda.synchronize()
            want = ref.bfloat16().float() * (h.float() if epi == 2 else 1.0)
            d = (c.float() - want).abs()
            bad = (d > 0.05 * want.abs().max()).nonzero()
            nbad_tot += len(bad)
            for rr, cc in bad[:4].tolist():
                print(f"epi{epi} sm{sm} it{it}: [{rr},{cc}] tile ({rr // 256},{cc // 256}) in-tile ({rr % 256},{cc % 256}) "
                      f"c={c[rr, cc].item():.4g} want={want[rr, cc].item():.4g} D={h[rr, cc].item():.4g} "
                      f"acc_true={ref[rr, cc].item():.4g} c/D={c[rr, cc].item() / (h[rr, cc].item() or 1):.4g}", flush=True)
        print(f"epi{epi} sm{sm}: total bad {nbad_tot} over 10 launches", flush=True)
