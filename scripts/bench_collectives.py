#!/usr/bin/env python
"""Collective bandwidth sweep over the fluxmpi_amd communicator (the nccl-tests analogue).

For each collective and message size: the mean time of ``--iters`` back-to-back calls after
``--warmup``, the algorithm bandwidth (bytes / time) and the bus bandwidth (the per-link rate
an ideal ring needs: x 2(N-1)/N for allreduce, x (N-1)/N for allgather / reduce-scatter /
alltoall, x 1 for broadcast) — the numbers to size DDP gradient buckets against on a node
(``parallel/ddp.py``: bucket_mb, first_bucket_mb, tail_bucket_mb). One JSON line per
(collective, size) on rank 0; max time over ranks.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/bench_collectives.py --sizes 1K,64K,1M,4M,16M,64M,256M
    python scripts/bench_collectives.py --device cpu        # gloo, plumbing check

Every rank runs the same sequence of collectives (SPMD); sizes are bytes of the send buffer
(bf16 elements by default).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

_BUS = {"allreduce": lambda n: 2.0 * (n - 1) / n, "allgather": lambda n: (n - 1) / n,
        "reduce_scatter": lambda n: (n - 1) / n, "alltoall": lambda n: (n - 1) / n, "broadcast": lambda n: 1.0}


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(s[-1:], 1)
    return int(float(s[:-1] if s[-1:] in "KMG" else s) * mult)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4K,64K,1M,4M,16M,64M")
    ap.add_argument("--ops", default="allreduce,allgather,reduce_scatter,broadcast,alltoall")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    args = ap.parse_args(argv)

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel import runtime

    FluxMPI.Init()
    rank, world = FluxMPI.local_rank(), FluxMPI.total_workers()
    use_cuda = args.device == "cuda" or (args.device == "auto" and torch.cuda.is_available())
    dev = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[args.dtype]
    if dev.type == "cpu" and dt != torch.float32:
        dt = torch.float32  # gloo reduces fp32
    esz = torch.empty((), dtype=dt).element_size()
    probe = torch.empty(1, dtype=dt, device=dev)
    comm = runtime.comm_for(probe)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for op in [o for o in args.ops.split(",") if o]:
        for s in args.sizes.split(","):
            nbytes = parse_size(s)
            n = max(world, nbytes // esz // world * world)  # divisible by the world for the scatter ops
            buf = torch.ones(n, dtype=dt, device=dev)
            if op == "allreduce":
                call = lambda: comm.allreduce(buf)  # noqa: E731
            elif op == "broadcast":
                call = lambda: comm.broadcast(buf, 0)  # noqa: E731
            elif op == "allgather":
                inp = buf[: n // world].clone()
                out = torch.empty(n, dtype=dt, device=dev)
                call = lambda: comm.allgather(out, inp)  # noqa: E731
            elif op == "reduce_scatter":
                out = torch.empty(n // world, dtype=dt, device=dev)
                call = lambda: comm.reduce_scatter(out, buf)  # noqa: E731
            elif op == "alltoall":
                out = torch.empty_like(buf)
                call = lambda: comm.alltoall(out, buf)  # noqa: E731
            else:
                raise SystemExit(f"unknown collective {op!r}")
            for _ in range(args.warmup):
                call()
            sync()
            FluxMPI.barrier()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                call()
            sync()
            t = (time.perf_counter() - t0) / args.iters
            t = FluxMPI.allreduce(torch.tensor([t], dtype=torch.float64), max).item() if world > 1 else t
            size = n * esz
            algbw = size / t / 1e9
            if rank == 0:
                print(json.dumps({"op": op, "bytes": size, "dtype": str(dt).replace("torch.", ""), "world": world,
                                  "backend": comm.name, "device": dev.type, "us": round(t * 1e6, 2),
                                  "algbw_GBps": round(algbw, 3), "busbw_GBps": round(algbw * _BUS[op](world), 3)}),
                      flush=True)
    FluxMPI.Finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
