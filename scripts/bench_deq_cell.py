#!/usr/bin/env python
"""The fused DEQ cell kernels (deq_cell.hip) at the MNIST DEQ shape (256 x 28 x 28 x 48, bf16
channels_last): us per forward (solver evaluation, out only) and per adjoint VJP with the fused
update, plus the outputs' max difference against the unfused 5-launch path. Run once per
FLUXMPI_DEQ_CELL_FWD_WAVES / FLUXMPI_DEQ_CELL_VJP_WAVES setting (read once per process)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluxmpi_amd.models.deq import ResidualCell  # noqa: E402
from fluxmpi_amd.ops import deq_cell  # noqa: E402


def t_us(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    torch.manual_seed(0)
    cell = ResidualCell(48).cuda()
    for p in cell.parameters():
        p.data = p.data.to(torch.bfloat16)
    cell = cell.to(memory_format=torch.channels_last)
    shp = (256, 48, 28, 28)
    z = torch.randn(shp, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x = torch.randn(shp, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    u = torch.randn(shp, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.randn(shp, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    _, state = deq_cell.cell_forward(cell, z, x, keep=True)
    fwd = t_us(lambda: deq_cell.cell_forward(cell, z, x))
    vjp = t_us(lambda: deq_cell.cell_vjp(cell, state, u, grad=g))
    # against the unfused path
    deq_cell.ENABLED = False
    ref = cell.forward_raw(z, x)
    _, st2 = cell.forward_state(z, x)
    ref_v = cell.vjp(st2, u)
    deq_cell.ENABLED = True
    got = deq_cell.cell_forward(cell, z, x)
    got_v = deq_cell.cell_vjp(cell, state, u)
    ef = float((got.float() - ref.float()).abs().max() / ref.float().abs().max())
    ev = float((got_v.float() - ref_v.float()).abs().max() / ref_v.float().abs().max())
    print(json.dumps({"fwd_waves": os.environ.get("FLUXMPI_DEQ_CELL_FWD_WAVES", "8"),
                      "vjp_waves": os.environ.get("FLUXMPI_DEQ_CELL_VJP_WAVES", "8"),
                      "fwd_us": round(fwd, 2), "vjp_us": round(vjp, 2), "fwd_rel_max_err": ef, "vjp_rel_max_err": ev}),
          flush=True)


if __name__ == "__main__":
    main()
