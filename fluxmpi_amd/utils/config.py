"""Configuration: persisted preferences + environment knobs.

Reference behaviour (``src/FluxMPI.jl:16-56``):

* a Preferences.jl key ``FluxMPIDisableCUDAMPISupport`` in
  ``LocalPreferences.toml`` read once at module init, written by
  ``disable_cudampi_support(; disable=true)`` and only effective after a
  restart;
* the removed env var ``FLUXMPI_DISABLE_CUDAMPI_SUPPORT`` only triggers a
  deprecation warning.

Here the preference lives in a TOML file (``$FLUXMPI_PREFS`` or
``./LocalPreferences.toml``) under ``[fluxmpi_amd]``. On MI355X the comm path
is RCCL and always device-direct; setting the preference re-creates the
reference's *host-staged* data path (GPU tensor -> host -> collective ->
device) which is useful only as an A/B/debug mode.

Environment knobs (all optional):

=========================  ==================================================
``FLUXMPI_BACKEND``        ``auto`` (default) | ``rccl`` (native C++ RCCL
                           communicator) | ``torch`` (torch.distributed
                           ProcessGroup) | ``gloo`` (CPU) | ``gloo-device``
                           (GPU compute, gloo collectives on device tensors:
                           several ranks on one GPU, which RCCL refuses)
``FLUXMPI_BUCKET_MB``      gradient bucket size in MiB (default 16)
``FLUXMPI_FIRST_BUCKET_MB`` size of the first (last-layer) bucket (default 4)
``FLUXMPI_COMM_DTYPE``     ``native`` | ``fp32`` | ``bf16`` grad comm dtype
``FLUXMPI_OVERLAP``        ``1`` (default) overlap allreduce with backward
``FLUXMPI_PROFILE``        ``1`` emit roctx ranges + per-step timers
``FLUXMPI_DEBUG_CHECKS``   ``1`` cross-rank checksum after every collective
``FLUXMPI_TIMEOUT_S``      collective watchdog timeout (default 600)
``FLUXMPI_FORCE_COMM``     ``1``: issue the collectives even in a world of
                           one (hooks, packing, RCCL on the comm stream), to
                           exercise and time the N>1 path on a single GPU
``FLUXMPI_DIRECT_GRADS``   ``1`` (default): the package's weight-gradient kernels
                           write straight into the DDP buckets (``ops/graddst``)
``FLUXMPI_OVERLAP_OPT``    ``1``: the DDP engine updates each bucket as soon as its
                           reduced gradient exists (comm stream / side stream),
                           during the rest of backward; ``0`` (default): in
                           ``step()``
=========================  ==================================================
"""
from __future__ import annotations

import logging
import os
import warnings
from dataclasses import dataclass, field

try:  # py3.11+
    import tomllib as _toml_reader  # type: ignore
except ModuleNotFoundError:  # pragma: no cover - py3.10 path
    try:
        import tomli as _toml_reader  # type: ignore
    except ModuleNotFoundError:  # pragma: no cover
        _toml_reader = None

log = logging.getLogger("fluxmpi_amd")

PREF_SECTION = "fluxmpi_amd"
PREF_DISABLE_KEY = "FluxMPIDisableCUDAMPISupport"


def prefs_path() -> str:
    return os.environ.get("FLUXMPI_PREFS", os.path.join(os.getcwd(), "LocalPreferences.toml"))


def _read_prefs(path: str) -> dict:
    if not os.path.exists(path) or _toml_reader is None:
        return {}
    with open(path, "rb") as f:
        try:
            data = _toml_reader.load(f)
        except Exception:  # malformed file: behave as if absent
            return {}
    return dict(data.get(PREF_SECTION, {}))


def _write_prefs(path: str, values: dict) -> None:
    """Minimal TOML writer for a flat ``[fluxmpi_amd]`` table (keeps other tables)."""
    other: dict = {}
    if os.path.exists(path) and _toml_reader is not None:
        with open(path, "rb") as f:
            try:
                other = _toml_reader.load(f)
            except Exception:
                other = {}
    other.pop(PREF_SECTION, None)
    merged = dict(_read_prefs(path))
    merged.update(values)

    def fmt(v):
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (int, float)):
            return repr(v)
        return '"' + str(v).replace('"', '\\"') + '"'

    lines = []
    for sec, tbl in other.items():
        if isinstance(tbl, dict):
            lines.append(f"[{sec}]")
            lines.extend(f"{k} = {fmt(v)}" for k, v in tbl.items() if not isinstance(v, dict))
            lines.append("")
    lines.append(f"[{PREF_SECTION}]")
    lines.extend(f"{k} = {fmt(v)}" for k, v in merged.items())
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def disable_cudampi_support(disable: bool = True) -> None:
    """Persist the "host-staged collectives" preference (reference ``src/FluxMPI.jl:51-56``).

    Like the reference, the change only takes effect in a *new* process.
    """
    _write_prefs(prefs_path(), {PREF_DISABLE_KEY: bool(disable)})
    log.info(
        "Device-direct (RCCL) collectives %s. Restart the process for this change to take effect!",
        "disabled" if disable else "enabled",
    )


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def _env_float(name: str, default: float) -> float:
    v = os.environ.get(name)
    try:
        return float(v) if v not in (None, "") else default
    except ValueError:
        return default


@dataclass
class Config:
    backend: str = "auto"
    host_staged: bool = False  # reference's CUDA-unaware path (Q1), debug only
    bucket_mb: float = 16.0
    first_bucket_mb: float = 4.0
    tail_bucket_mb: float = 2.0  # the last-closing bucket is tapered to this (0: off), ddp._taper
    comm_dtype: str = "native"
    overlap: bool = True
    profile: bool = False
    debug_checks: bool = False
    timeout_s: float = 600.0
    force_comm: bool = False
    direct_grads: bool = True  # ops write parameter gradients into their DDP bucket slices
    overlap_opt: bool = False  # per-bucket optimiser update during backward (DDP)
    # cross-rank structure check of functional reduction plans: always / first / never
    check_plans: str = "always"
    # gradient-bucket sizes at N > 1: "auto" (measured unless sizes are given explicitly),
    # "measured" (probe the communicator: parallel/bucket_plan.py), "default" (the sizes above)
    bucket_plan: str = "auto"
    buckets_explicit: bool = False  # a bucket size came from the environment or the preferences
    extra: dict = field(default_factory=dict)

    @classmethod
    def load(cls) -> "Config":
        if "FLUXMPI_DISABLE_CUDAMPI_SUPPORT" in os.environ:
            warnings.warn(
                "FLUXMPI_DISABLE_CUDAMPI_SUPPORT environment variable has been removed and has no "
                "effect. Please use `fluxmpi_amd.disable_cudampi_support()` instead.",
                stacklevel=2,
            )
        prefs = _read_prefs(prefs_path())
        return cls(
            backend=os.environ.get("FLUXMPI_BACKEND", prefs.get("backend", "auto")).lower(),
            host_staged=bool(prefs.get(PREF_DISABLE_KEY, False)),
            bucket_mb=_env_float("FLUXMPI_BUCKET_MB", float(prefs.get("bucket_mb", 16.0))),
            first_bucket_mb=_env_float("FLUXMPI_FIRST_BUCKET_MB", float(prefs.get("first_bucket_mb", 4.0))),
            tail_bucket_mb=_env_float("FLUXMPI_TAIL_BUCKET_MB", float(prefs.get("tail_bucket_mb", 2.0))),
            comm_dtype=os.environ.get("FLUXMPI_COMM_DTYPE", prefs.get("comm_dtype", "native")).lower(),
            overlap=_env_bool("FLUXMPI_OVERLAP", bool(prefs.get("overlap", True))),
            profile=_env_bool("FLUXMPI_PROFILE", False),
            debug_checks=_env_bool("FLUXMPI_DEBUG_CHECKS", False),
            timeout_s=_env_float("FLUXMPI_TIMEOUT_S", 600.0),
            force_comm=_env_bool("FLUXMPI_FORCE_COMM", bool(prefs.get("force_comm", False))),
            direct_grads=_env_bool("FLUXMPI_DIRECT_GRADS", bool(prefs.get("direct_grads", True))),
            overlap_opt=_env_bool("FLUXMPI_OVERLAP_OPT", bool(prefs.get("overlap_opt", False))),
            check_plans=os.environ.get("FLUXMPI_CHECK_PLANS", str(prefs.get("check_plans", "always"))).lower(),
            bucket_plan=os.environ.get("FLUXMPI_BUCKET_PLAN", str(prefs.get("bucket_plan", "auto"))).lower(),
            buckets_explicit=any(os.environ.get(k) for k in ("FLUXMPI_BUCKET_MB", "FLUXMPI_FIRST_BUCKET_MB",
                                                             "FLUXMPI_TAIL_BUCKET_MB"))
            or any(k in prefs for k in ("bucket_mb", "first_bucket_mb", "tail_bucket_mb")),
            extra=prefs,
        )


_CONFIG: Config | None = None


def get_config(reload: bool = False) -> Config:
    global _CONFIG
    if _CONFIG is None or reload:
        _CONFIG = Config.load()
    return _CONFIG
