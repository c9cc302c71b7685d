#!/usr/bin/env python
"""Cost of the cross-rank plan check of the functional API (parallel/optimizer.py check_plan) on the
host group: 2 gloo ranks, the ResNet-50 gradient tree's structure (161 leaves), `always` vs the
`like=`-derived once-per-plan check. usage: python scripts/bench_check_plan.py -> JSON lines."""
import json
import os
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.models import resnet50
    from fluxmpi_amd.parallel.optimizer import check_plan

    FluxMPI.Init()
    tree = {n: torch.zeros(1) for n, _ in resnet50().named_parameters()}  # the structure only
    res = {}
    for name, derived in (("always", False), ("like_derived", True)):
        for _ in range(20):
            check_plan(tree, "bench", derived=derived)
        FluxMPI.barrier()
        t0 = time.perf_counter()
        n = 500
        for _ in range(n):
            check_plan(tree, "bench", derived=derived)
        res[name + "_us_per_call"] = round(1e6 * (time.perf_counter() - t0) / n, 2)
    if rank == 0:
        q.put(res)
    FluxMPI.Finalize()


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, 29611, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join()
    print(json.dumps({"bench": "check_plan", "world": 2, "backend": "gloo (host)", "leaves": 161, **out}))
