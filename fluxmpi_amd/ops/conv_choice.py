"""Per-shape kernel choices of the convolution paths, measured once per shape on first use (the
analogue of cudnn.benchmark / MIOpen's find-db; the reference leaves this to cuDNN through Flux,
``/root/reference/src/FluxMPI.jl`` has no kernel selection of its own).

Tables (key -> choice), shipped / exchanged as JSON lines (``dump_choices`` / ``load_choices``,
``bench.py --choices``, ``parallel/autotune.calibrate`` broadcasts rank 0's so every rank runs
the same kernels):

================  ================================================================
``_FWD1_CHOICE``  1x1 forward: our GEMM + statistics epilogue (True) or MIOpen
``_FWD_CHOICE``   3x3 / s1 forward: ours (True) or MIOpen; ``_FWD_ENGINE`` our tile config
``_S2_CHOICE``    3x3 / s2 forward: ours + statistics epilogue (True) or MIOpen
``_DS_CHOICE``    downsample 1x1 forward: ours + statistics epilogue (True) or MIOpen
``_DGRAD_CHOICE`` 3x3 / s1 input gradient with narrow channels: ours (True) or MIOpen
``_WG_CHOICE``    weight gradients: ("miopen" | "ours" | "w256" | "w3n", our kernel config)
``_LB_CHOICE``    token-major Linear backward in one launch (linbwd.hip): split count
================  ================================================================

Frozen (``freeze_choices``) or inside a HIP-graph capture, a missing shape takes the
deterministic default instead of a timing that could differ between ranks.
"""
from __future__ import annotations

import os

import torch

from . import _ext
from . import gemm as G
from . import graddst

# weight gradients of the bottleneck convolutions: "auto" = the fastest (measured once per
# shape) of MIOpen and our split-K transposed-operand kernel in a few configurations
WGRAD = "auto"
# our 3x3 forward tile configurations: 0: auto (128x128 tiles); 8 / 7: 256x128 tiles, 64- / 32-deep K-steps
FWD_ENGINES = (0, 8, 7)
# our weight-gradient kernel configurations tried by the autotune: (variant, target workgroups); s44 sweep
_WG_CONFIGS = ((2, 512), (2, 768), (2, 1024), (2, 384))
# the narrow 3x3 weight-gradient kernel (wgrad3x3n.hip) configurations: (variant, target workgroups);
# variant bit 0: 8 waves (else 4), bit 1 (4 waves only): the next two blocks in flight (else one)
_W3N_CONFIGS = ((1, 256), (2, 256), (0, 256), (1, 512))
# ... for the 128-channel layers (bit 2: 128 output channels per workgroup)
_W3N_CONFIGS_128 = ((5, 256), (4, 256), (1, 256), (5, 512))


def w3n_configs(ci: int):
    """The wgrad3x3n configurations the autotune times for ``ci`` input channels."""
    return _W3N_CONFIGS_128 if ci == 128 else _W3N_CONFIGS
# the statistics pass a MIOpen forward then needs is priced at one read of the output at this rate
_STATS_PASS_BPS = 5e12

_FWD1_CHOICE: dict = {}
_FWD_CHOICE: dict = {}
_FWD_ENGINE: dict = {}
_S2_CHOICE: dict = {}
_DS_CHOICE: dict = {}
_DGRAD_CHOICE: dict = {}
_WG_CHOICE: dict = {}
_LB_CHOICE: dict = {}
_CHOICE_TABLES = {"linbwd_splits": "_LB_CHOICE", "fwd1x1_ours": "_FWD1_CHOICE", "fwd3x3_ours": "_FWD_CHOICE", "wgrad": "_WG_CHOICE",
                  "fwd_ds_ours": "_DS_CHOICE", "fwd3x3s2_ours": "_S2_CHOICE", "fwd3x3_engine": "_FWD_ENGINE",
                  "dgrad3x3_ours": "_DGRAD_CHOICE"}

_FROZEN = False


def no_measure() -> bool:
    """Take the default instead of timing: inside a HIP-graph capture, or once frozen."""
    return _FROZEN or torch.cuda.is_current_stream_capturing()


def time_us(fn, iters=10, repeats=3):
    """Best of ``repeats`` timings of ``iters`` back-to-back calls (choices flip on single-sample
    noise otherwise)."""
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(repeats):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def linbwd_choice(key, candidates, default: int, run) -> int:
    """The split count of a Linear's one-launch backward (``ops/linear.dgrad_wgrad``) for ``key``:
    the fastest of ``candidates`` (``run(splits)`` launches the kernel into scratch buffers),
    measured once per shape; ``default`` when frozen / capturing."""
    hit = _LB_CHOICE.get(key)
    if hit is not None:
        return hit
    if no_measure():
        return default
    with torch.no_grad():
        best = min(candidates, key=lambda sp: time_us(lambda: run(sp), iters=5, repeats=3))
    _LB_CHOICE[key] = best
    return best


def stats_choice(table: dict, key, make) -> bool:
    """Our kernel with the next BatchNorm's statistics in its epilogue vs MIOpen plus the
    statistics pass over its output; measured once per key. ``make()`` (called only to measure)
    returns (ours, theirs, output bytes)."""
    hit = table.get(key)
    if hit is not None:
        return hit
    if no_measure():
        return True
    with torch.no_grad():
        ours, theirs, out_bytes = make()
        t_ours = time_us(ours)
        t_theirs = time_us(theirs)
    table[key] = t_ours <= t_theirs + out_bytes / _STATS_PASS_BPS * 1e6
    return table[key]


def w256_ok(co: int, ci: int, dc: torch.Tensor) -> bool:
    """The 256x256-tile weight-gradient kernel (wgrad256.hip) takes both widths and enough rows."""
    if dc.dtype != torch.bfloat16:
        return False
    C = _ext.get(required=True)
    k = dc.numel() // co
    return bool(C.wgrad256_supported(co, ci, k, co, ci)) and k >= 4096


def _with_cfg(cfg, fn):
    saved = G.WGRAD_VARIANT, G.WGRAD_TARGET_WG
    G.WGRAD_VARIANT, G.WGRAD_TARGET_WG = cfg
    try:
        return fn()
    finally:
        G.WGRAD_VARIANT, G.WGRAD_TARGET_WG = saved


def wgrad_best(key, impls: dict, param=None):
    """Run the fastest weight-gradient implementation for ``key`` (measured on first use: MIOpen
    vs our kernel in each of ``_WG_CONFIGS``, "w256" when offered, and "w3n" — a callable taking one
    of ``_W3N_CONFIGS`` — when offered) and return its result.
    ``param``: the weight, whose DDP bucket slice (if any) receives the returned gradient
    (``graddst``; never during the measurements)."""
    choice = _WG_CHOICE.get(key)
    if choice is None:
        if WGRAD == "miopen" or no_measure():
            choice = ("miopen", None)
        elif WGRAD == "ours":
            choice = ("ours", _WG_CONFIGS[0])
        else:
            best = (time_us(impls["miopen"]), ("miopen", None))
            for cfg in _WG_CONFIGS:
                t = _with_cfg(cfg, lambda: time_us(impls["ours"]))
                if t < best[0]:
                    best = (t, ("ours", cfg))
            if "w256" in impls:
                t = time_us(impls["w256"])
                if t < best[0]:
                    best = (t, ("w256", None))
            if "w3n" in impls:
                for cfg in impls.get("w3n_cfgs", _W3N_CONFIGS):
                    t = time_us(lambda: impls["w3n"](cfg))
                    if t < best[0]:
                        best = (t, ("w3n", cfg))
            choice = best[1]
        _WG_CHOICE[key] = choice
    name, cfg = choice
    with graddst.into(param):
        if name == "w3n":
            return impls[name](cfg)
        return impls[name]() if cfg is None else _with_cfg(cfg, impls[name])


def dump_choices():
    """The per-shape choices measured so far, as JSON-lines records (``scripts/show_choices.py``)."""
    import json
    g = globals()
    return [json.dumps({"kind": kind, "key": str(k), "choice": str(v)})
            for kind, name in _CHOICE_TABLES.items() for k, v in g[name].items()]


def load_choice_lines(lines) -> int:
    """Pre-populate the tables from JSON-lines records (``dump_choices``): those shapes skip the
    first-step measurement (no autotune time, no run-to-run flips of marginal shapes); others are
    still measured (unless frozen). Returns the entries loaded."""
    import ast
    import json
    g = globals()
    n = 0
    for line in lines:
        line = line.strip()
        if not line:
            continue
        rec = json.loads(line)
        name = _CHOICE_TABLES.get(rec["kind"])
        if name is None:
            continue
        g[name][ast.literal_eval(rec["key"])] = ast.literal_eval(rec["choice"])
        n += 1
    return n


def load_choices(path: str) -> int:
    """:func:`load_choice_lines` from a file."""
    with open(path) as f:
        return load_choice_lines(f.readlines())


def freeze_choices(frozen: bool = True) -> None:
    """Stop measuring (``parallel/autotune.calibrate``: rank-consistent tables at N > 1)."""
    global _FROZEN
    _FROZEN = frozen


def choices_frozen() -> bool:
    return _FROZEN


if os.environ.get("FLUXMPI_KERNEL_CHOICES"):
    load_choices(os.environ["FLUXMPI_KERNEL_CHOICES"])
