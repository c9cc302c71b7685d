"""Debug: EPI 2 split with D = 1 (c = bf16(acc)) vs EPI 0 split; dump a bad row's pattern."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from fluxmpi_amd.ops import _ext

C = _ext.get(required=True)
st = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
m, n, k = 50432, 768, 2304
a = ((torch.rand(m, k, device="cuda") * 2 - 1)).bfloat16()
w = ((torch.rand(n, k, device="cuda") * 2 - 1) * k ** -0.5).bfloat16()
ones = torch.ones(m, n, device="cuda", dtype=torch.bfloat16)
part = torch.zeros(C.gemm_nt_colpart_rows(m), n, device="cuda")
C.gemm_nt_set_split(8)
c0 = torch.zeros(m, n, device="cuda", dtype=torch.bfloat16)
C.gemm_nt(a.data_ptr(), w.data_ptr(), c0.data_ptr(), 0, 0, 0, 0, 0, k, k, n, m, n, k, 0, st)
torch.cuda.synchronize()
ref = (a.float() @ w.float().t())
print("epi0 split max err", float((c0.float() - ref).abs().max()))
for it in range(12):
    c = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
    part.zero_()
    C.gemm_nt(a.data_ptr(), w.data_ptr(), c.data_ptr(), 0, 0, 0, ones.data_ptr(), part.data_ptr(), k, k, n, m, n, k, 2, st)
    torch.cuda.synchronize()
    d = (c.float() - c0.float()).abs()
    bad = (d > 0.05).nonzero()
    # colpart rows: 2 * tile_m + wr (fp32 column sums of the rounded dh over 128 rows)
    pr = part.view(-1, 2, n).sum(1)  # per tile_m
    cs = c0.float().view(-1, 256, n).sum(1)
    perr = float((pr - cs).abs().max())
    print(f"it{it}: nbad {len(bad)} colpart max err {perr:.4g}", flush=True)
    if len(bad):
        r0 = int(bad[0, 0])
        row = c[r0].float()
        exp = c0[r0].float()
        t0 = int(bad[0, 1]) // 256 * 256
        badc = [cc for cc in range(t0, t0 + 256) if abs(row[cc] - exp[cc]) > 0.05]
        print(f"  row {r0} (in-tile {r0 % 256}) tile_n {t0 // 256}: bad cols (in-tile) {[cc - t0 for cc in badc]}")
        print("  got ", [round(float(row[cc]), 4) for cc in badc[:12]])
        print("  want", [round(float(exp[cc]), 4) for cc in badc[:12]])
        # is the neighbourhood the raw bits of fp32 values? show raw u16 of 8 around the first bad
        cb = badc[0] // 8 * 8
        raw = c[r0, cb:cb + 8].view(torch.int16).tolist()
        print("  raw16 chunk", cb - t0, [hex(x & 0xffff) for x in raw])
        print("  want chunk", [round(float(x), 4) for x in exp[cb:cb + 8]])
