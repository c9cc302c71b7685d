"""Which Python lines launch the DEQ step's PyTorch (non-HIP-extension) kernels: one training step
under torch.profiler (record_shapes + stacks), aten ops grouped by (op, shape, innermost repo frame)."""
import collections
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models import build_model
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    dev = FluxMPI.device()
    model = build_model("deq").to(dev, memory_format=torch.channels_last)
    for m in model.modules():
        if not isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    ddp = DDP(model, O.Adam(1e-3), average=True)
    x = torch.randn(256, 1, 28, 28, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (256,), device=dev)

    def step():
        loss = F.cross_entropy(ddp(x).float(), y)
        loss.backward()
        ddp.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], record_shapes=True,
                                with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    table = prof.key_averages(group_by_input_shape=True, group_by_stack_n=6)
    rows = sorted(table, key=lambda e: -e.count)
    for e in rows[:40]:
        if e.key in ("aten::empty", "aten::empty_strided", "aten::view", "aten::as_strided", "aten::detach"):
            continue
        stack = " <- ".join(f for f in (e.stack or []) if "fluxmpi" in f or "bench" in f or "models" in f)[:300]
        print(f"{e.count:5d}  {e.key:28s} {str(e.input_shapes)[:48]:50s} {stack}")


if __name__ == "__main__":
    main()
