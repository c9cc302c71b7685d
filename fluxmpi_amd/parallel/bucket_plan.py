"""Measured gradient-bucket plan: probe the live communicator, fit it, size the buckets from the fit.

The engine's buckets (``parallel/ddp.py``) trade two costs of a ring allreduce over xGMI:

* every collective pays a fixed latency ``alpha`` (launch, ring set-up, the per-step hand-offs:
  tens of microseconds for RCCL over 8 ranks), so small buckets waste the links;
* a bucket is launched only when its last gradient exists, and the bucket that closes last (the
  first layers) runs entirely after the backward, so large buckets hold traffic back and expose
  it.

Both are properties of the communicator actually in use — RCCL over the node's xGMI mesh, RCCL
with fewer ranks, gloo on the host — so instead of fixed sizes the plan comes from a measurement:
:func:`probe` times an allreduce ladder (256 KiB .. 64 MiB of the gradient dtype) on the live
communicator, every rank takes the slowest rank's time per size (the collective finishes with
its slowest member), :func:`fit` fits ``t(n) = alpha + beta * n`` (relative least squares) and
:func:`choose` sizes the buckets from the fit's half-performance message size
``n_half = alpha / beta`` (the bytes at which latency and transfer cost the same):

* ``bucket``  = 4 ``n_half``: each full bucket moves at >= 80 % of the asymptotic bus bandwidth;
* ``first``   = 2 ``n_half``: the first gradients leave early, at >= 67 %;
* ``tail``    = 1 ``n_half``: the exposed last piece costs ~2 ``alpha`` (the taper of
  ``DDP._taper`` grows from it towards the front);

clamped to [0.25, 64] MiB and to at most 64 buckets over the model's gradient bytes. Rank 0's
choice is broadcast, so every rank builds the same plan. The measured samples and the
fit travel into the bench record (``DDP.comm_summary()``: ``comm_probe``, ``bucket_plan``), so the
first run on a new topology returns the per-size bus bandwidth it saw.

Reference: ``/root/reference/src/optimizer.jl:45-65`` issues one collective per gradient leaf, all
at once; the bucket sizes here decide how those leaves are grouped on the wire.
"""
from __future__ import annotations

import json
import math
import time
from dataclasses import dataclass

import torch

MIB = 1 << 20
LADDER = (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20)
MIN_BYTES, MAX_BYTES = MIB // 4, 64 * MIB


@dataclass
class CommModel:
    """``t(n) = alpha_us + beta_us_per_byte * n`` for an allreduce of ``n`` bytes over ``world`` ranks."""
    alpha_us: float
    beta_us_per_byte: float
    world: int

    def time_us(self, nbytes: float) -> float:
        return self.alpha_us + self.beta_us_per_byte * nbytes

    def n_half(self) -> float:
        """Message size at which latency and transfer cost the same (bytes)."""
        return self.alpha_us / self.beta_us_per_byte if self.beta_us_per_byte > 0 else float("inf")

    def busbw_gbs(self, nbytes: float | None = None) -> float:
        """Bus bandwidth (ring-allreduce convention: 2 (W - 1) / W bytes per byte) in GB/s, at
        ``nbytes`` or asymptotically."""
        f = 2.0 * (self.world - 1) / self.world if self.world > 1 else 1.0
        if nbytes is None:
            return f / self.beta_us_per_byte / 1e3 if self.beta_us_per_byte > 0 else float("inf")
        return f * nbytes / self.time_us(nbytes) / 1e3


def fit(samples: list[tuple[int, float]], world: int) -> CommModel:
    """Least squares of ``t = alpha + beta n`` on relative error (each sample weighted by 1 / t, so
    the small sizes, which carry ``alpha``, count as much as the large ones); ``alpha >= 0``,
    ``beta > 0``."""
    pts = [(float(n), float(t)) for n, t in samples if n > 0 and t > 0]
    if len(pts) < 2:
        raise ValueError("bucket_plan.fit: need at least two (bytes, us) samples")
    # minimise sum ((alpha + beta n - t) / t)^2  ->  2x2 normal equations in (alpha, beta)
    s11 = sum(1.0 / t ** 2 for n, t in pts)
    s12 = sum(n / t ** 2 for n, t in pts)
    s22 = sum(n * n / t ** 2 for n, t in pts)
    r1 = sum(1.0 / t for n, t in pts)
    r2 = sum(n / t for n, t in pts)
    det = s11 * s22 - s12 * s12
    alpha, beta = ((r1 * s22 - r2 * s12) / det, (s11 * r2 - s12 * r1) / det) if det > 0 else (0.0, 0.0)
    if beta <= 0 or alpha < 0:
        # degenerate ladders (noise, a flat curve): the largest message's rate, and the smallest
        # message's time as the latency
        nmax, tmax = max(pts)
        beta = max(tmax / nmax, 1e-12)
        alpha = max(0.0, min(pts)[1] - beta * min(pts)[0])
        if alpha == 0.0:
            beta = max(min(t / n for n, t in pts), 1e-12)
    return CommModel(alpha, beta, world)


def _quantise(nbytes: float, up: bool = False) -> int:
    """Round (``up``: up) to a multiple of 0.25 MiB inside [MIN_BYTES, MAX_BYTES]."""
    q = MIB // 4
    k = math.ceil(nbytes / q) if up else round(nbytes / q)
    return int(min(MAX_BYTES, max(MIN_BYTES, k * q)))


def choose(model: CommModel, total_bytes: int | None = None, max_buckets: int = 64) -> dict:
    """Bucket sizes (MiB) from the fitted model (module docstring)."""
    nh = model.n_half()
    if not math.isfinite(nh):
        nh = MAX_BYTES
    bucket = _quantise(4 * nh, up=True)  # up: the >= 80 % promise holds after rounding
    if total_bytes:
        bucket = max(bucket, _quantise(total_bytes / max_buckets))
    first = min(_quantise(2 * nh), bucket)
    tail = min(_quantise(nh), first)
    return {"bucket_mb": bucket / MIB, "first_bucket_mb": first / MIB, "tail_bucket_mb": tail / MIB,
            "n_half_mb": round(nh / MIB, 3), "alpha_us": round(model.alpha_us, 2),
            "busbw_gbs": round(model.busbw_gbs(), 2)}


def probe(comm, device: torch.device, dtype: torch.dtype = torch.bfloat16, sizes=LADDER, iters: int = 5,
          warmup: int = 2, cpu_comm=None, passes: int = 2) -> list[tuple[int, float]]:
    """Time ``comm.allreduce`` over the ``sizes`` ladder (bytes) of ``dtype``; returns
    ``[(bytes, us)]`` with each time the MAXIMUM over ranks (identical on every rank). Host wall
    time around ``iters`` back-to-back collectives, the device synchronised at both ends (the
    collective's own stream included); the ladder runs ``passes`` times and each size keeps its
    fastest pass (a rank arriving late at the first timed size inflated it ~6x in the gloo
    rehearsals, profiles/rd6ai_rehearsals.jsonl)."""
    esz = torch.empty((), dtype=dtype).element_size()
    buf = torch.zeros(max(sizes) // esz, dtype=dtype, device=device)
    cuda = device.type == "cuda"
    best: dict = {}
    for _ in range(max(1, passes)):
        for nb in sizes:
            t = buf[: max(1, nb // esz)]
            for _ in range(warmup):
                comm.allreduce(t)
            if cuda:
                torch.cuda.synchronize(device)
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                comm.allreduce(t)
            if cuda:
                torch.cuda.synchronize(device)
            us = (time.perf_counter() - t0) / iters * 1e6
            key = t.numel() * esz
            best[key] = min(us, best.get(key, float("inf")))
    out = list(best.items())
    del buf
    times = torch.tensor([us for _, us in out], dtype=torch.float64)
    if cpu_comm is not None and cpu_comm.size > 1:
        from .comm import ReduceOp
        cpu_comm.allreduce(times, ReduceOp.MAX)
    return [(nb, float(us)) for (nb, _), us in zip(out, times.tolist())]


def measured_plan(comm, device: torch.device, dtype: torch.dtype, total_bytes: int, cpu_comm=None,
                  root: int = 0) -> tuple[dict, list[dict]]:
    """Probe, fit and choose on every rank; rank ``root``'s plan is broadcast (host group).
    Returns ``(plan, samples)`` with ``samples = [{"kib", "us", "busbw_gbs"}]``."""
    from .autotune import broadcast_lines

    samples = probe(comm, device, dtype, cpu_comm=cpu_comm)
    model = fit(samples, comm.size)
    plan = choose(model, total_bytes)
    if cpu_comm is not None and cpu_comm.size > 1:
        plan = json.loads(broadcast_lines([json.dumps(plan)], root)[0])
    f = 2.0 * (comm.size - 1) / comm.size if comm.size > 1 else 1.0
    rec = [{"kib": nb >> 10, "us": round(us, 1), "busbw_gbs": round(f * nb / us / 1e3, 2)} for nb, us in samples]
    return plan, rec


__all__ = ["CommModel", "fit", "choose", "probe", "measured_plan", "LADDER"]
