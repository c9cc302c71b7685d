"""``DistributedDataContainer`` (reference ``src/data.jl:1-26``).

Splits any indexable dataset (``len`` + ``__getitem__``; a ``torch.utils.data.Dataset``,
a tensor, a numpy array, a list ...) into contiguous per-rank shards with the
reference's formula:

    size_per_process = ceil(len(data) / world)
    partitions = [range(i, min(i + size_per_process, len)) for i in range(0, len, size_per_process)]
    idxs = partitions[rank]

so every rank but the last holds ``ceil(len/world)`` items and the last holds
the remainder. When the formula yields fewer partitions than ranks (e.g.
``len=10, world=6``) the reference throws a ``BoundsError``; we
raise a ``ValueError`` that explains why.
"""
from __future__ import annotations

import math
from typing import Any

import numpy as np
import torch

from . import runtime


class DistributedDataContainer(torch.utils.data.Dataset):
    """Rank-local contiguous shard of ``data`` (also a ``torch.utils.data.Dataset``)."""

    def __init__(self, data: Any, rank: int | None = None, world: int | None = None):
        total = len(data)
        world = runtime.total_workers() if world is None else world
        rank = runtime.local_rank() if rank is None else rank
        per = int(math.ceil(total / world)) if total else 0
        if per == 0:
            raise ValueError("DistributedDataContainer: cannot shard an empty dataset")
        starts = list(range(0, total, per))
        if rank >= len(starts):
            raise ValueError(
                f"DistributedDataContainer: {total} items split in blocks of {per} give only "
                f"{len(starts)} partitions for {world} ranks (rank {rank} would get none)")
        lo = starts[rank]
        self.data = data
        self.idxs = range(lo, min(lo + per, total))

    def __len__(self) -> int:
        return len(self.idxs)

    def _map(self, i):
        if isinstance(i, slice):
            return list(self.idxs[i])
        if isinstance(i, (list, tuple, np.ndarray, torch.Tensor)):
            return [self.idxs[int(j)] for j in (i.tolist() if hasattr(i, "tolist") else i)]
        return self.idxs[int(i)]

    def __getitem__(self, i):
        j = self._map(i)
        if isinstance(j, list):
            if isinstance(self.data, (torch.Tensor, np.ndarray)):
                return self.data[j]
            return [self.data[k] for k in j]
        return self.data[j]

    def __iter__(self):
        for k in range(len(self)):
            yield self[k]

    # MLUtils interface names
    def numobs(self) -> int:
        return len(self)

    def getobs(self, i):
        return self[i]
