"""Race / divergence detection and failure detection.

The reference has neither: a rank whose gradient tree differs simply hangs in
``MPI_Allreduce``, and a dead rank aborts the job through MPI's
default error handler. Here:

* :func:`check_replicas` — cross-rank checksum (fp64 sum and sum of squares)
  of a model / tree of tensors; raises :class:`ReplicaDivergenceError` when
  ranks disagree (e.g. a missed ``synchronize`` or a non-deterministic
  update). With ``FLUXMPI_DEBUG_CHECKS=1`` the DDP engine runs it after
  every optimiser step.
* :func:`check_same_structure` — allgather of a structure hash: raises
  :class:`~fluxmpi_amd.utils.errors.CollectiveMismatchError` *before* a
  bucketed collective when ranks would issue different collectives.
* :class:`Watchdog` — a daemon thread that polls the device communicator
  for asynchronous RCCL errors and for collectives that stay incomplete
  longer than ``FLUXMPI_TIMEOUT_S``; on failure it aborts the communicator
  (so blocked ranks return instead of hanging) and records the error, which
  :meth:`Watchdog.check` re-raises on the training thread.
"""
from __future__ import annotations

import hashlib
import threading
import time
import weakref

import torch

from .errors import CollectiveMismatchError
from .tree import leaves, structure_signature


class ReplicaDivergenceError(RuntimeError):
    pass


def _tensors_of(obj) -> list:
    if isinstance(obj, torch.nn.Module):
        return [p.detach() for p in obj.parameters()] + [b.detach() for b in obj.buffers()]
    return [t for t in leaves(obj) if isinstance(t, torch.Tensor)]


def checksum(obj) -> torch.Tensor:
    """fp64 ``[sum, sum_sq, numel]`` over all tensors of ``obj`` (on CPU)."""
    s = torch.zeros(3, dtype=torch.float64)
    for t in _tensors_of(obj):
        if t.numel() == 0 or not (t.is_floating_point() or t.dtype in (torch.int32, torch.int64)):
            continue
        d = t.double()
        s[0] += d.sum().item()
        s[1] += (d * d).sum().item()
        s[2] += t.numel()
    return s


def check_replicas(obj, rtol: float = 0.0, comm=None) -> None:
    """Raise if ``obj`` is not identical (within ``rtol``) on every rank."""
    from ..parallel import runtime

    c = comm or runtime.cpu_comm()
    if c.size == 1:
        return
    mine = checksum(obj)
    hi, lo = mine.clone(), mine.clone()
    c.allreduce(hi, "max")
    c.allreduce(lo, "min")
    scale = torch.maximum(hi.abs(), lo.abs()).clamp_min(1e-300)
    if bool(((hi - lo).abs() > rtol * scale).any()):
        raise ReplicaDivergenceError(f"replicas diverged: checksum range min={lo.tolist()} max={hi.tolist()} "
                                     f"(rank {c.rank} has {mine.tolist()})")


def structure_hash(obj) -> int:
    sig = structure_signature(obj).encode()
    return int.from_bytes(hashlib.sha1(sig).digest()[:7], "little")


def check_same_structure(obj, comm=None, what: str = "tree") -> None:
    """Raise :class:`CollectiveMismatchError` if ranks hold differently shaped trees."""
    from ..parallel import runtime

    c = comm or runtime.cpu_comm()
    if c.size == 1:
        return
    mine = structure_hash(obj)
    # one collective: max of (h, -h) gives the max and (minus) the min at once
    hl = torch.tensor([mine, -mine], dtype=torch.int64)
    c.allreduce(hl, "max")
    hi, lo = int(hl[0]), -int(hl[1])
    h = mine
    if hi != lo:
        raise CollectiveMismatchError(f"ranks disagree about the structure of the {what} "
                                      f"(rank {c.rank} hash {int(h)}); collectives would mismatch")


_WATCHDOGS: "weakref.WeakSet[Watchdog]" = weakref.WeakSet()


class Watchdog:
    """Background failure detector for the device communicator.

    Each poll runs under ``_poll_lock``; :meth:`pause` takes the same lock, so
    once it returns no poll is running and none starts until :meth:`resume`.
    HIP-graph capture needs that (an event query from another thread is illegal
    while a stream captures), and :func:`stop_all` (``Finalize``) stops every
    watchdog before the communicator is destroyed, so the thread can never poll
    a freed communicator.
    """

    def __init__(self, comm, timeout_s: float = 600.0, interval_s: float = 1.0):
        self.comm = comm
        self.timeout_s = timeout_s
        self.interval_s = interval_s
        self.error: BaseException | None = None
        self._inflight: dict = {}
        self._lock = threading.Lock()
        self._poll_lock = threading.Lock()
        self._paused = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="fluxmpi-watchdog", daemon=True)
        _WATCHDOGS.add(self)
        self._thread.start()

    def track(self, work, what: str = "collective"):
        """Register an in-flight :class:`Work`; returns it."""
        if self._paused:
            return work  # captured into a graph: nothing runs now, nothing to watch
        with self._lock:
            self._inflight[id(work)] = (work, time.time(), what)
        return work

    def _poll(self):
        self.comm.check_async_error()
        now = time.time()
        with self._lock:
            items = list(self._inflight.items())
        for k, (w, t0, what) in items:
            if w.is_completed():
                with self._lock:
                    self._inflight.pop(k, None)
            elif now - t0 > self.timeout_s:
                raise TimeoutError(f"{what} did not complete within {self.timeout_s:.0f}s")

    def _run(self):
        while not self._stop.wait(self.interval_s):
            with self._poll_lock:
                if self._paused or self._stop.is_set():
                    continue
                try:
                    self._poll()
                except BaseException as e:  # noqa: BLE001 - recorded and re-raised on the main thread
                    self.error = e
                    self._abort(repr(e))
                    return

    def _abort(self, reason: str):
        abort = getattr(self.comm, "abort", None)
        try:
            if abort is not None:
                abort(f"watchdog: {reason}")
            else:
                h = getattr(self.comm, "_h", None)
                if h is not None and hasattr(h, "abort"):
                    h.abort()
        except Exception:
            pass

    def pause(self):
        """Stop polling (returns once no poll is running); forget in-flight works."""
        with self._poll_lock:
            self._paused = True
            with self._lock:
                self._inflight.clear()

    def resume(self):
        with self._poll_lock:
            self._paused = False

    def check(self):
        if self.error is not None:
            raise RuntimeError(f"communicator failure detected by watchdog: {self.error!r}") from self.error

    def stop(self):
        self._stop.set()
        with self._poll_lock:  # wait for a running poll to end
            pass
        if self._thread is not threading.current_thread():
            self._thread.join(timeout=5)


def stop_all() -> None:
    """Stop every live watchdog (``Finalize`` calls this before destroying communicators)."""
    for w in list(_WATCHDOGS):
        w.stop()


__all__ = ["ReplicaDivergenceError", "CollectiveMismatchError", "checksum", "check_replicas", "structure_hash",
           "check_same_structure", "Watchdog", "stop_all"]
