"""Checkpoint / resume (absent in the reference; the documented way to
share optimiser state is ``synchronize!(opt_state)`` from the root after setup).

``save(path, tree)`` writes from ``root_rank`` only (parameters, optimiser
state trees with :class:`~fluxmpi_amd.optimisers.Leaf` nodes, DDP state
dicts, Python scalars) in a format readable by
``torch.load(weights_only=True)``: tensors are moved to CPU and every
container is converted to plain dicts / lists with type tags.

``load(path, like=None)`` reads on every rank (``map_location`` = this rank's
device) and, when ``like`` is given, copies values in place into the live
tree so views (e.g. the DDP engine's flat buckets) stay valid. Follow with
``synchronize(..., root_rank)`` if only the root can see the file.
"""
from __future__ import annotations

import os

import torch

from .tree import node_def

_TAG = "__fluxmpi_node__"


def _encode(x):
    from ..optimisers import Leaf

    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, Leaf):
        return {_TAG: "Leaf", "rule": repr(x.rule), "state": _encode(x.state), "frozen": x.frozen}
    if isinstance(x, torch.nn.Module):
        return {_TAG: "Module", "state": {k: v.detach().cpu() for k, v in x.state_dict().items()}}
    if isinstance(x, (bool, int, float, complex, str)) or x is None:
        return x
    if isinstance(x, tuple) and hasattr(x, "_fields"):
        return {_TAG: "namedtuple", "fields": list(x._fields), "values": [_encode(v) for v in x]}
    if isinstance(x, tuple):
        return {_TAG: "tuple", "values": [_encode(v) for v in x]}
    if isinstance(x, list):
        return [_encode(v) for v in x]
    if isinstance(x, dict):
        return {str(k): _encode(v) for k, v in x.items()}
    nd = node_def(x)
    if nd is not None:
        ch, _ = nd[0](x)
        return {_TAG: "node", "type": type(x).__name__, "values": [_encode(c) for c in ch]}
    raise TypeError(f"checkpoint: cannot encode {type(x)}")


def _decode(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device)
    if isinstance(x, list):
        return [_decode(v, device) for v in x]
    if isinstance(x, dict):
        tag = x.get(_TAG)
        if tag == "tuple":
            return tuple(_decode(v, device) for v in x["values"])
        if tag == "namedtuple":
            return dict(zip(x["fields"], (_decode(v, device) for v in x["values"])))
        if tag == "Leaf":
            return {"rule": x["rule"], "state": _decode(x["state"], device), "frozen": x["frozen"]}
        if tag == "Module":
            return {k: v.to(device) for k, v in x["state"].items()}
        if tag == "node":
            return [_decode(v, device) for v in x["values"]]
        return {k: _decode(v, device) for k, v in x.items()}
    return x


def save(path: str, obj, root_rank: int = 0) -> None:
    """Write ``obj`` from ``root_rank`` (all ranks may call; others return after a barrier)."""
    from ..parallel import runtime

    rank = runtime.local_rank() if runtime.Initialized() else 0
    if rank == root_rank:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(_encode(obj), tmp)
        os.replace(tmp, path)
    if runtime.Initialized() and runtime.total_workers() > 1:
        runtime.barrier()


def load(path: str, like=None, device=None):
    """Load a checkpoint (``weights_only=True``). With ``like``, copy into it in place and return it."""
    from ..optimisers import Leaf
    from ..parallel import runtime

    dev = device or (runtime.device() if runtime.Initialized() else torch.device("cpu"))
    raw = torch.load(path, map_location="cpu", weights_only=True)
    data = _decode(raw, dev)
    if like is None:
        return data

    def copy_into(dst, src):
        if isinstance(dst, torch.nn.Module):
            dst.load_state_dict(src)
            return dst
        if isinstance(dst, torch.Tensor):
            with torch.no_grad():
                dst.copy_(src)
            return dst
        if isinstance(dst, Leaf):
            dst.state = copy_into(dst.state, src["state"])
            dst.frozen = src["frozen"]
            return dst
        nd = node_def(dst)
        if nd is None:
            return src
        ch, aux = nd[0](dst)
        if isinstance(src, dict) and not isinstance(dst, dict):
            src_vals = list(src.values())
        elif isinstance(src, dict):
            src_vals = [src[str(k)] for k in dst.keys()]
        else:
            src_vals = list(src)
        return nd[1](aux, [copy_into(d, s) for d, s in zip(ch, src_vals)])

    return copy_into(like, data)
