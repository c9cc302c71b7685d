#!/usr/bin/env python
"""Probe: can two ranks share one MI355X through the native RCCL communicator?

Launch: ``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
--master-port P scripts/probe_two_ranks_one_gpu.py``. Both ranks pin ``cuda:0``
(``gpu_devices=[0, 0]``), bootstrap ``RcclComm`` through the store (the
``ncclUniqueId`` exchange of ``parallel/comm.py``) and allreduce one tensor.
Each rank prints one JSON line with the outcome (or the exact error).
"""
import json
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import fluxmpi_amd as FluxMPI

    rank = int(os.environ.get("RANK", "0"))
    rec = {"rank": rank, "probe": "rccl-two-ranks-one-gpu"}
    try:
        FluxMPI.Init(gpu_devices=[0, 0], backend="rccl")
        t = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
        FluxMPI.allreduce(t, "+")
        torch.cuda.synchronize()
        rec.update(ok=True, backend=FluxMPI.backend_name(), value=float(t[0].item()), expect=3.0)
    except Exception as e:  # noqa: BLE001 - the error text is the probe's result
        rec.update(ok=False, error=f"{type(e).__name__}: {e}", tb=traceback.format_exc()[-2000:])
    print(json.dumps(rec), flush=True)
    try:
        FluxMPI.Finalize()
    except Exception:
        pass


if __name__ == "__main__":
    main()
