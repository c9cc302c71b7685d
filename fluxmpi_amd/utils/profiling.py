"""Tracing / profiling (the reference has none; users time with ``time()``).

* :func:`range` — a roctx range (shows up in ``rocprofv3 --marker-trace`` and
  in ``rocprofv3 --kernel-trace`` timelines) around a region; no-op when
  ``libroctx64`` is not loadable or ``FLUXMPI_PROFILE`` is off.
* :class:`StepTimer` — per-phase GPU time of a training step measured with
  HIP events on the compute stream (``fwd``/``bwd``/``comm_wait``/``opt``),
  aggregated over steps; ``summary()`` returns means in ms.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

import torch

from .config import get_config

_ROCTX = None
_TRIED = False


def _roctx():
    global _ROCTX, _TRIED
    if _TRIED:
        return _ROCTX
    _TRIED = True
    cands = []
    try:
        cands.append(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:
        pass
    cands += ["/opt/rocm/lib/libroctx64.so", "libroctx64.so"]
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _ROCTX = lib
            break
        except OSError:
            continue
    return _ROCTX


def enabled() -> bool:
    return get_config().profile


@contextlib.contextmanager
def range(name: str, force: bool = False):  # noqa: A001 - mirrors roctx naming
    lib = _roctx() if (force or enabled()) else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx() if enabled() else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class StepTimer:
    """Accumulate GPU time per named phase using HIP events (CPU wall time on CPU)."""

    def __init__(self, device: torch.device | None = None):
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.totals: dict = {}
        self.counts: dict = {}
        self._pending: list = []

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.device.type == "cuda":
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            with range(name):
                yield
            e.record()
            self._pending.append((name, s, e))
        else:
            t0 = time.perf_counter()
            yield
            self._add(name, (time.perf_counter() - t0) * 1e3)

    def _add(self, name, ms):
        self.totals[name] = self.totals.get(name, 0.0) + ms
        self.counts[name] = self.counts.get(name, 0) + 1

    def flush(self):
        if self._pending:
            torch.cuda.synchronize(self.device)
            for name, s, e in self._pending:
                self._add(name, s.elapsed_time(e))
            self._pending.clear()

    def summary(self) -> dict:
        self.flush()
        return {k: self.totals[k] / self.counts[k] for k in self.totals}

    def reset(self):
        self.flush()
        self.totals.clear()
        self.counts.clear()
