"""Stress check of gemm_nt's epilogues (store-data hazard hunt): repeated launches of EPI 1 (bias +
GELU and its derivative) and EPI 2 (GELU backward) on 591-tile shapes with the split tail on and off;
counts wrong / non-finite elements against fp32 references. FLUXMPI_C_VARIANT selects a build."""
import os
import sys
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 1)[0])
import load_variant  # noqa: E402
load_variant.install()
from fluxmpi_amd.ops import _ext  # noqa: E402
from fluxmpi_amd.ops import gelu as GL  # noqa: E402

C = _ext.get(required=True)
GL.set_form("tanh")
GL._sync(C)
st = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
reps = int(os.environ.get("REPS", "10"))
tot = {}
for (m, n, k) in [(50432, 768, 2304), (50432, 3072, 768), (50432, 768, 3072)]:
    a = ((torch.rand(m, k, device="cuda") * 2 - 1)).bfloat16()
    w = ((torch.rand(n, k, device="cuda") * 2 - 1) * k ** -0.5).bfloat16()
    bias = (torch.randn(n, device="cuda") * 0.5).float()
    h = ((torch.rand(m, n, device="cuda") * 2 - 1)).bfloat16()
    acc = a.float() @ w.float().t()
    y = (acc + bias).bfloat16().float()
    ref_d, ref_g = GL._gelu_grad_ref(y), GL.gelu(y)
    ref_dh = acc.bfloat16().float() * h.float()
    part = torch.zeros(C.gemm_nt_colpart_rows(m), n, device="cuda")
    for sm in (8, 0):
        C.gemm_nt_set_split(sm)
        for epi in (1, 2):
            bad = 0
            for _ in range(reps):
                c = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
                c2 = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
                C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), c2.data_ptr() if epi == 1 else 0,
                          bias.data_ptr() if epi == 1 else 0, 1, h.data_ptr() if epi == 2 else 0,
                          part.data_ptr() if epi == 2 else 0, k, k, n, m, n, k, epi, st)
                torch.cuda.synchronize()
                outs = [(c, ref_d), (c2, ref_g)] if epi == 1 else [(c, ref_dh)]
                for got, ref in outs:
                    e = (got.float() - ref).abs()
                    bad += int((~torch.isfinite(got.float())).sum()) + int((e > 0.05 * ref.abs().max()).sum())
            key = f"m{m}n{n}k{k} split{sm} epi{epi}"
            tot[key] = bad
            print(f"{key}: wrong elements over {reps} launches: {bad}", flush=True)
        del c, c2
    del a, w, h, acc, y, ref_d, ref_g, ref_dh
    torch.cuda.empty_cache()
print("TOTAL wrong:", sum(tot.values()))
