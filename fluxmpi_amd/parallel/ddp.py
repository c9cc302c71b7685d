"""``DDP``: the high-performance data-parallel training engine.

This is what the reference's step loop (per-leaf blocking,
host-staged allreduce inside ``Optimisers.update``) becomes when designed
for MI355X + RCCL over xGMI:

1. **Flat bucket views.** At construction every trainable parameter is moved
   into a contiguous per-bucket buffer and ``p.data`` / ``p.grad`` become
   strided views into it (channels_last weights keep their strides). Autograd
   then accumulates gradients straight into the communication buffer: there
   is no pack/unpack on the hot path and the optimiser runs over a few large
   flat buffers.
2. **Buckets in backward order.** Buckets are filled from the last parameter
   to the first (the order autograd produces gradients); the first bucket is
   small (``first_bucket_mb``, 4 MiB) so communication starts early, the rest
   are ``bucket_mb`` (16 MiB). Sizing: a ring allreduce over xGMI is per-link
   bound and pays ~10-30 us per collective, so buckets must be MBs; but the
   bucket that closes last (the first layers) is fully exposed after
   backward, and in a CNN most parameters sit in the LAST stages (ResNet-50:
   ~30 of 51 MB in layer4), so a 64 MiB bucket would hold back almost all
   traffic until backward ends. 16 MiB gives 4-5 bf16 buckets for ResNet-50,
   all but ~3 MB of them overlapped with the rest of backward.
3. **Backward/comm overlap.** A post-accumulate-grad hook per parameter counts
   down its bucket; a full bucket is allreduced immediately on the
   communicator's own HIP stream (fenced by an event recorded on
   the compute stream). Buckets are launched strictly in index order on every
   rank, so collectives can never be mismatched across ranks.
4. **Fused optimiser.** ``step()`` waits per bucket and runs one fused
   multi-tensor HIP kernel per bucket (Adam/AdamW/Descent/Momentum/Nesterov
   with Optimisers.jl numerics; optional fp32 master weights for bf16
   models). Step-dependent scalars (``beta^t``) live on the device, so the
   whole step can be captured in a HIP graph.
5. **Semantics.** Gradients are SUMmed like the reference; ``average=True``
   scales by ``1/world`` inside the optimiser kernel (free).
6. **World of one.** With nothing to communicate (world 1) the engine neither
   registers hooks nor packs: the fused optimiser reads autograd's gradient
   tensors in place (pointer lists, no copy into the flat buffer).
   ``force_comm=True`` (``FLUXMPI_FORCE_COMM=1``) runs the full N>1 path
   anyway — hooks, packing, real collectives on the communicator's stream
   with event fencing — so a single GPU exercises and measures it.

The Optimisers.jl-compatible state tree is available via
:meth:`DDP.optimiser_state` (``Leaf(rule, (mt, vt, βt))`` with tensor views
into the flat moment buffers).
"""
from __future__ import annotations

import os
import weakref
from contextlib import contextmanager
from dataclasses import dataclass, field

import torch

from .. import optimisers as O
from ..ops import multi_tensor as mt
from ..ops import _ext
from ..ops import graddst
from ..ops import optim as fused
from ..utils.config import get_config
from ..utils import profiling
from ..utils.debug import Watchdog, check_replicas, check_same_structure
from . import runtime
from .comm import Communicator, ReduceOp


# module -> weakref to its engine: the engine holds the module strongly, so a strong value here
# would keep every engine ever built (model, flat buffers, masters, moments) alive for good
_ENGINES: "weakref.WeakKeyDictionary[torch.nn.Module, weakref.ref]" = weakref.WeakKeyDictionary()


def engine_for(module: torch.nn.Module) -> "DDP | None":
    """The DDP engine managing ``module`` (None if there is none, or it was discarded)."""
    ref = _ENGINES.get(module)
    return ref() if ref is not None else None


@dataclass
class _Bucket:
    index: int
    dtype: torch.dtype
    device: torch.device
    params: list
    offsets: list
    numel: int
    flat_param: torch.Tensor | None = None
    flat_grad: torch.Tensor | None = None
    master: torch.Tensor | None = None
    exp_avg: torch.Tensor | None = None
    exp_avg_sq: torch.Tensor | None = None
    pending: int = 0
    ready: bool = False
    launched: bool = False
    packed: bool = False
    work: object = None
    names: list = field(default_factory=list)
    comm_buf: torch.Tensor | None = None
    carry: torch.Tensor | None = None
    applied: bool = False  # overlap_opt: this step's update already enqueued (during backward)


def _strided_view(flat: torch.Tensor, like: torch.Tensor, offset: int) -> torch.Tensor:
    """A view of ``flat[offset:offset+numel]`` with ``like``'s sizes and (dense) strides."""
    return flat.as_strided(like.size(), like.stride(), flat.storage_offset() + offset)


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and the same strides on every dimension of size > 1 (memory order)."""
    return a.shape == b.shape and all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def _is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (contiguous under some dim permutation)."""
    if t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last):
        return True
    dims = sorted(range(t.dim()), key=lambda d: t.stride(d))
    expect = 1
    for d in dims:
        if t.size(d) != 1 and t.stride(d) != expect:
            return False
        expect *= t.size(d)
    return True


class DDP:
    """Data-parallel wrapper: ``loss = ddp(x)...; loss.backward(); ddp.step()``.

    Parameters
    ----------
    module: the model (already on its device, in its compute dtype/memory format).
    rule:   an ``optimisers`` rule (Adam, AdamW chain, Descent, Momentum, Nesterov);
            the engine runs it with fused flat-buffer kernels.
    master_weights: keep fp32 master copies (+ fp32 moments) for low-precision params.
    average: divide the summed gradient by the world size (default False = reference SUM).
    overlap: launch bucket allreduces from backward hooks (default: ``FLUXMPI_OVERLAP``).
    broadcast: synchronise parameters and buffers from ``root_rank`` at construction.
    overlap_opt: per-bucket optimiser overlap (default ``FLUXMPI_OVERLAP_OPT``): as soon as a
            bucket's gradients are complete (and, when communicating, its allreduce is enqueued)
            its fused update is enqueued behind it — on the communicator's in-order stream, or on
            a side stream at world 1 — instead of after the whole backward in ``step()``. Safe
            because a bucket is complete only after every backward node that reads its
            parameters has run (a parameter's post-accumulate hook fires once, after all its
            uses); ``step()`` then only fences. Contract: every backward that completes buckets
            is followed by ``step()`` (no inspection of reduced-but-unapplied gradients).
    """

    def __init__(self, module: torch.nn.Module, rule: O.AbstractRule | None = None, *,
                 bucket_mb: float | None = None, first_bucket_mb: float | None = None,
                 master_weights: bool = True, average: bool = False, overlap: bool | None = None,
                 broadcast: bool = True, root_rank: int = 0, comm: Communicator | None = None,
                 comm_dtype: torch.dtype | None = None, watchdog: bool | None = None,
                 grad_mode: str | None = None, force_comm: bool | None = None,
                 tail_bucket_mb: float | None = None, overlap_opt: bool | None = None):
        cfg = get_config()
        # "steal": autograd hands over each freshly produced gradient (no in-place accumulate
        # kernel per parameter, no zero fill) and one multi-tensor launch per bucket packs them
        # into the flat buffer; "view": p.grad is a view into the flat buffer (autograd adds in).
        self.grad_mode = grad_mode or cfg.extra.get("grad_mode", "steal")
        if self.grad_mode not in ("steal", "view"):
            raise ValueError(f"DDP: grad_mode must be 'steal' or 'view', got {self.grad_mode!r}")
        self.module = module
        self.rule = rule if rule is not None else O.Adam()
        self.average = average
        self.overlap = cfg.overlap if overlap is None else overlap
        self.master_weights = master_weights
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("DDP: module has no trainable parameters")
        self.device = params[0].device
        if comm is None:
            comm = runtime.comm_for(params[0]) if runtime.Initialized() else None
        self.comm = comm
        self.world = comm.size if comm is not None else 1
        self.force_comm = cfg.force_comm if force_comm is None else bool(force_comm)
        if self.force_comm and comm is None:
            raise RuntimeError("DDP(force_comm=True) needs a communicator: call fluxmpi_amd.Init() first")
        # collectives are issued whenever there is a peer, or when forced (world-1 rehearsal)
        self.communicate = comm is not None and (self.world > 1 or self.force_comm)
        # measurement tool (FLUXMPI_EMULATE_COMM="WGS:GBPS[:THREADS[:LDS_KB]]"): with each bucket's
        # collective, hold WGS workgroups (THREADS threads, LDS_KB of LDS each) on the comm stream
        # for the time a ring allreduce of the bucket would take at GBPS bus bandwidth on 8
        # ranks — RCCL's CU footprint, which a world of one lacks
        self._emulate = None
        emu = cfg.extra.get("emulate_comm") or os.environ.get("FLUXMPI_EMULATE_COMM", "")
        if emu and self.communicate and self.device.type == "cuda":
            f = emu.split(":")
            self._emulate = (int(f[0]), float(f[1]), int(f[2]) if len(f) > 2 else 256,
                             int(f[3]) * 1024 if len(f) > 3 else 0)
        if comm_dtype is None:
            comm_dtype = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
                          "bfloat16": torch.bfloat16, "fp16": torch.float16}.get(cfg.comm_dtype)
        self.comm_dtype = comm_dtype
        # measured bucket plan (parallel/bucket_plan.py): at N > 1, unless sizes were given
        self.bucket_plan, self.comm_probe = "default", None
        explicit = bucket_mb is not None or first_bucket_mb is not None or tail_bucket_mb is not None \
            or cfg.buckets_explicit
        if self.communicate and self.world > 1 and (cfg.bucket_plan == "measured"
                                                    or (cfg.bucket_plan == "auto" and not explicit)):
            from . import bucket_plan as BP
            nbytes: dict = {}
            for p in params:
                nbytes[p.dtype] = nbytes.get(p.dtype, 0) + p.numel() * p.element_size()
            wire = comm_dtype or max(nbytes, key=nbytes.get)
            plan, rec = BP.measured_plan(comm, self.device, wire, sum(nbytes.values()),
                                         cpu_comm=runtime.cpu_comm() if runtime.Initialized() else None)
            bucket_mb, first_bucket_mb, tail_bucket_mb = plan["bucket_mb"], plan["first_bucket_mb"], plan["tail_bucket_mb"]
            self.bucket_plan, self.comm_probe = "measured", {"samples": rec, "plan": plan}
        bb = int((bucket_mb if bucket_mb is not None else cfg.bucket_mb) * (1 << 20))
        fb = int((first_bucket_mb if first_bucket_mb is not None else cfg.first_bucket_mb) * (1 << 20))
        tb = int((tail_bucket_mb if tail_bucket_mb is not None else cfg.tail_bucket_mb) * (1 << 20))
        names = {id(p): n for n, p in module.named_parameters()}
        self.buckets = self._build_buckets(params, bb, fb, names, tb)
        self._param_bucket = {}
        for b in self.buckets:
            for p in b.params:
                self._param_bucket[id(p)] = b
        # direct delivery ("steal" mode with collectives): the package's weight-gradient kernels
        # allocate each parameter's gradient in its bucket slice (ops/graddst.py), so the
        # per-bucket pack finds it in place (the pack was one copy kernel per bucket)
        self.direct_grads = bool(cfg.direct_grads) and self.communicate and self.grad_mode == "steal"
        for b in self.buckets:
            for p, o in zip(b.params, b.offsets):
                if self.direct_grads:
                    graddst.attach(p, b.flat_grad, o)
                else:
                    graddst.detach(p)  # a previous engine's buckets are not this one's
        self._hooks = []
        self._sync_enabled = True
        # per-bucket optimiser overlap: on the communicator's in-order stream (behind the bucket's
        # allreduce) when it has one, on a side stream when nothing is communicated, else in
        # step() (host-synchronous collectives: nothing to overlap with)
        want_opt = cfg.overlap_opt if overlap_opt is None else bool(overlap_opt)
        self.overlap_opt = want_opt and self.overlap and self.grad_mode == "steal"
        self._opt_stream = None  # None: the update runs right after the (host-waited) reduction
        if self.overlap_opt and self.device.type == "cuda":
            if not self.communicate:
                self._opt_stream = torch.cuda.Stream(self.device)
            elif getattr(comm, "in_order", False) and getattr(comm, "stream", None) is not None:
                self._opt_stream = comm.stream
        if self.overlap and (self.communicate or self.overlap_opt):
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad_ready))
        self._setup_optimizer()
        self.debug_checks = cfg.debug_checks
        self.watchdog = None
        if self.world > 1 and runtime.Initialized():
            # every rank must build the same bucket plan, or collectives would mismatch
            check_same_structure([(str(b.dtype), b.numel, len(b.params)) for b in self.buckets],
                                 comm=runtime.cpu_comm(), what="DDP bucket plan")
        if self.communicate and runtime.Initialized():
            if watchdog if watchdog is not None else cfg.extra.get("watchdog", True):
                self.watchdog = Watchdog(comm, timeout_s=cfg.timeout_s)
        if broadcast and self.communicate:
            self.broadcast_parameters(root_rank)
        self._next_launch = 0
        self._direct_cache: dict = {}
        self._views: dict = {}
        self._record_versions()
        self._carry_live = False
        self._carry_hook = None
        self.collectives_launched = 0  # gradient-bucket allreduces issued so far
        self.pack_copies = 0  # gradients the bucket packs had to copy (not delivered in place)
        self.pack_copied: dict = {}  # shape -> copies (which producers still miss their slices)
        _ENGINES[module] = weakref.ref(self)
        self.zero_grad()
        self.step_count = 0
        # exposed-communication timing (off by default: event timing costs a little)
        self.timing = bool(cfg.profile)
        self._comm_events: list = []

    # ------------------------------------------------------------------ setup
    @staticmethod
    def _taper(group: list, esz: int, tail_bytes: int) -> list:
        """Split the bucket that closes LAST (the first layers: their gradients come at the very
        end of backward, so its whole allreduce is exposed) into pieces that grow geometrically
        towards the front: from the end, at most tail, 2 tail, 4 tail, ... bytes. The layers
        before the final tail then launch mid-backward and only ``tail_bytes`` stay exposed
        (ResNet-50's last 14 MB bucket mixed layer3, ready mid-backward,
        with layer1 / stem)."""
        out, cur, cur_bytes, cap = [], [], 0, tail_bytes
        for p in reversed(group):  # from the parameter whose gradient comes last
            nb = p.numel() * esz
            if cur and cur_bytes + nb > cap:
                out.append(list(reversed(cur)))
                cur, cur_bytes, cap = [], 0, cap * 2
            cur.append(p)
            cur_bytes += nb
        if cur:
            out.append(list(reversed(cur)))
        out.reverse()
        if len(out) > 1 and sum(p.numel() for p in out[0]) * esz < tail_bytes:
            out[1] = out[0] + out[1]  # no sliver bucket at the front: one collective fewer
            out.pop(0)
        return out

    def _build_buckets(self, params, bucket_bytes, first_bytes, names, tail_bytes=0):
        rev = list(reversed(params))
        by_dtype: dict = {}
        for p in rev:
            by_dtype.setdefault(p.dtype, []).append(p)
        buckets: list[_Bucket] = []
        for dt, ps in by_dtype.items():
            esz = torch.empty((), dtype=dt).element_size()
            groups, cur, cur_bytes = [], [], 0
            limit = first_bytes
            for p in ps:
                nb = p.numel() * esz
                if cur and cur_bytes + nb > limit:
                    groups.append(cur)
                    cur, cur_bytes, limit = [], 0, bucket_bytes
                cur.append(p)
                cur_bytes += nb
            if cur:
                groups.append(cur)
            if tail_bytes > 0 and len(groups) > 1:
                groups = groups[:-1] + self._taper(groups[-1], esz, tail_bytes)
            for g in groups:
                buckets.append(self._make_bucket(len(buckets), dt, g, names))
        # launch order = expected completion order: a bucket is ready when its LAST parameter
        # (in backward order) has its gradient. Ordering by the first parameter instead would
        # put a small bucket of another dtype (ResNet's fp32 BatchNorm parameters, spread over
        # the whole network) early in the sequence and hold every later bucket's allreduce
        # until the end of backward. Identical on every rank (built from the parameter list).
        order = {id(p): i for i, p in enumerate(rev)}
        buckets.sort(key=lambda b: max(order[id(p)] for p in b.params))
        for i, b in enumerate(buckets):
            b.index = i
        return buckets

    def _make_bucket(self, idx, dtype, params, names):
        for p in params:
            if not _is_dense(p):
                raise ValueError(f"DDP: parameter {names.get(id(p))} is not dense")
        offs, total = mt.aligned_offsets([p.numel() for p in params], dtype)
        dev = params[0].device
        flat_p = torch.zeros(total, dtype=dtype, device=dev)
        flat_g = torch.zeros(total, dtype=dtype, device=dev)
        with torch.no_grad():
            for p, o in zip(params, offs):
                v = _strided_view(flat_p, p, o)
                v.copy_(p.data)
                p.data = v
                if self.grad_mode == "view":
                    p.grad = _strided_view(flat_g, p, o)
        return _Bucket(idx, dtype, dev, list(params), offs, total, flat_p, flat_g,
                       names=[names.get(id(p), "?") for p in params])

    def _setup_optimizer(self):
        r = self.rule
        if isinstance(r, O.OptimiserChain) and len(r.opts) == 2 and isinstance(r.opts[0], O.Adam) \
                and isinstance(r.opts[1], O.WeightDecay):
            self.kind, self.adam, self.wd = "adam", r.opts[0], r.opts[1].gamma
        elif isinstance(r, O.Adam):
            self.kind, self.adam, self.wd = "adam", r, 0.0
        elif isinstance(r, O.Nesterov):
            self.kind, self.wd = "nesterov", 0.0
        elif isinstance(r, O.Momentum):
            self.kind, self.wd = "momentum", 0.0
        elif isinstance(r, O.Descent):
            self.kind, self.wd = "descent", 0.0
        else:
            raise TypeError(f"DDP: no fused kernel for rule {r!r}; use the functional optimisers API")
        dev = self.device
        for b in self.buckets:
            low = b.dtype in (torch.bfloat16, torch.float16)
            use_master = self.master_weights and low
            sdt = torch.float32 if use_master else b.dtype
            if use_master:
                b.master = b.flat_param.float()
            if self.kind == "adam":
                b.exp_avg = torch.zeros(b.numel, dtype=sdt, device=dev)
                b.exp_avg_sq = torch.zeros(b.numel, dtype=sdt, device=dev)
            elif self.kind in ("momentum", "nesterov"):
                b.exp_avg = torch.zeros(b.numel, dtype=sdt, device=dev)
        if self.kind == "adam":
            a = self.adam
            # device hyper block [lr, beta1^t, beta2^t]; beta^t starts at beta (Optimisers.jl init)
            self.hyper = torch.tensor([a.eta, a.beta[0], a.beta[1]], dtype=torch.float32, device=dev)
        else:
            self.hyper = torch.tensor([self.rule.eta], dtype=torch.float32, device=dev)

    def broadcast_parameters(self, root_rank: int = 0):
        """One broadcast per flat bucket (+ its fp32 master) + module buffers (``synchronize``
        of the model). Broadcasting the masters keeps them bit-identical on every rank."""
        if hasattr(self, "_versions"):
            self._sync_masters()  # the root's outside edits reach its master before it is sent
        with torch.no_grad():
            for b in self.buckets:
                self.comm.broadcast(b.flat_param, root_rank)
                if b.master is not None:
                    self.comm.broadcast(b.master, root_rank)
            # buffers and the parameters outside every bucket (requires_grad=False: a frozen
            # backbone or embedding) — the reference's synchronize! reaches every leaf
            bucketed = {id(p) for b in self.buckets for p in b.params}
            rest, seen = [], set()
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                if id(t) not in bucketed and id(t) not in seen and t.numel() > 0:
                    seen.add(id(t))
                    rest.append(t.detach())
            if rest:
                from .bucket import broadcast_tensors
                broadcast_tensors(rest, root_rank, comm=self.comm, force_comm=self.force_comm)
        if hasattr(self, "_versions"):
            self._record_versions()  # params and masters were written together: nothing stale

    # ------------------------------------------------------------------ hooks
    @contextmanager
    def no_sync(self):
        """Gradient accumulation: backward passes inside do not launch allreduces."""
        prev, self._sync_enabled = self._sync_enabled, False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _on_grad_ready(self, p):
        if not self._sync_enabled:
            return
        b = self._param_bucket[id(p)]
        if b.pending <= 0 or b.launched:
            # a second backward reached this bucket before step(): its first gradients are
            # already being reduced (and, with overlap_opt, applied to the weights the second
            # backward may have read) — accumulating into them would silently drop or corrupt
            # the update, so refuse loudly (accumulate under no_sync() instead)
            raise RuntimeError(
                f"DDP: a second backward reached gradient bucket {b.index} before step(); its "
                "gradients were already " + ("reduced and applied" if self.overlap_opt else "sent for reduction")
                + ". Accumulate gradients inside `with ddp.no_sync():` and run the last backward "
                "outside it, then step()")
        b.pending -= 1
        if b.pending == 0:
            b.ready = True
            self._launch_ready()

    def _launch_ready(self):
        while self._next_launch < len(self.buckets) and self.buckets[self._next_launch].ready:
            self._launch(self.buckets[self._next_launch])
            self._next_launch += 1

    def _launch(self, b: _Bucket):
        if b.launched:
            return
        b.launched = True
        if self.overlap_opt and not self._masters_synced:
            self._sync_masters()  # outside edits reach the masters before the step's first update
            self._masters_synced = True
        if self.communicate:
            self._launch_comm(b)
        if self.overlap_opt:
            self._apply_overlapped(b)

    def _apply_overlapped(self, b: _Bucket):
        """Enqueue bucket ``b``'s update now. Communicating: behind its allreduce on the in-order
        comm stream (stream order is the dependency: no fence, no host wait). World 1: on the
        side stream, after an event on the compute stream (the bucket's gradients are produced
        there) — the compute stream goes on with backward."""
        gscale = 1.0 / self.world if self.average else 1.0
        st = self._opt_stream
        if st is None:
            # no in-order device stream (CPU tensors, gloo on device tensors): wait for the
            # reduction here, then update on the current stream — the same order, no overlap
            if self.communicate:
                self._finish(b)
                self._add_carry(b)
                self._apply(b, gscale)
            elif not self._apply_direct(b, gscale):
                self._pack(b)
                self._apply(b, gscale)
            b.applied = True
            return
        if not self.communicate:
            st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            if self.communicate:
                if b.comm_buf is not None and self.comm_dtype != b.dtype:
                    mt.unpack(b.comm_buf, [b.flat_grad], [0])
                self._add_carry(b)
                self._apply(b, gscale)
            elif not self._apply_direct(b, gscale):
                self._pack(b)
                self._apply(b, gscale)
        b.applied = True

    def _launch_comm(self, b: _Bucket):
        self._pack(b)
        buf = b.flat_grad
        if self.comm_dtype is not None and self.comm_dtype != b.dtype:
            # K5: cast the bucket to the wire dtype (e.g. fp32 grads sent as bf16) in one launch
            if b.comm_buf is None:
                b.comm_buf = torch.empty(b.numel, dtype=self.comm_dtype, device=b.device)
            mt.pack([b.flat_grad], b.comm_buf, [0])
            buf = b.comm_buf
        with profiling.range(f"fluxmpi.allreduce.bucket{b.index}"):
            if self._emulate is not None and hasattr(self.comm, "stream"):
                wgs, gbps, thr, lds = self._emulate
                nbytes = buf.numel() * buf.element_size()
                us = 2.0 * 7.0 / 8.0 * nbytes / (gbps * 1e3)  # ring allreduce, 8 ranks
                self.comm.stream.wait_stream(torch.cuda.current_stream(self.device))
                _ext.get(required=True).emulate_comm(wgs, max(us, 5.0), self.comm.stream.cuda_stream, thr, lds)
            b.work = self.comm.allreduce(buf, ReduceOp.SUM, async_op=True)
        self.collectives_launched += 1
        if self.watchdog is not None:
            self.watchdog.track(b.work, f"allreduce of gradient bucket {b.index} ({b.numel} elements)")

    # ------------------------------------------------------------------ public
    def __call__(self, *args, **kw):
        return self.module(*args, **kw)

    forward = __call__

    def zero_grad(self):
        """Reset the gradients and re-arm the hooks. "view" mode zeroes the flat buffers (one
        fill launch per dtype); "steal" mode drops the per-step gradient tensors."""
        if self.grad_mode == "view":
            mt.fill_([b.flat_grad for b in self.buckets], 0.0)
        self._drop_carry()
        self._rearm()
        for b in self.buckets:
            for p, o in zip(b.params, b.offsets):
                if self.grad_mode == "steal":
                    p.grad = None
                elif p.grad is None or p.grad.data_ptr() != b.flat_grad.data_ptr() + o * b.flat_grad.element_size():
                    # someone replaced .grad (e.g. set_to_none): restore the view
                    p.grad = _strided_view(b.flat_grad, p, o)

    def _rearm(self):
        """Reset the per-step bucket state (countdowns, launch/pack flags) for the next backward."""
        for b in self.buckets:
            b.pending = len(b.params)
            b.ready = b.launched = b.packed = b.applied = False
            b.work = None
            if getattr(self, "direct_grads", False):
                for p in b.params:
                    graddst.rearm(p)
        self._next_launch = 0
        self._masters_synced = False

    def _note_copy(self, p) -> None:
        self.pack_copies += 1
        key = "x".join(str(d) for d in p.shape)
        self.pack_copied[key] = self.pack_copied.get(key, 0) + 1

    def _pack(self, b: _Bucket):
        """"steal" mode: copy the bucket's gradients into its flat buffer, one multi-tensor launch.

        Autograd's layout contract gives every gradient its parameter's (dense) strides, and the
        flat slice is a view with the same strides, so a raw copy of ``numel`` elements is exact.
        Parameters that received no gradient get zeros.
        """
        if self.grad_mode != "steal" or b.packed:
            return
        b.packed = True
        views = self._grad_views(b)
        srcs, dptrs, ns = [], [], []
        for p, dst, dptr in views:
            g = p.grad
            if g is None:
                dst.zero_()
            elif g.data_ptr() == dptr:
                if not _same_layout(g, dst):
                    dst.copy_(g.clone())
                    self._note_copy(p)
                # else already in place (delivered by the producing op, or p.grad set to the view)
            elif g.dtype is b.dtype and g.is_cuda and g.stride() == dst.stride():
                # the common case: autograd's layout contract (the parameter's dense strides)
                srcs.append(g)
                dptrs.append(dptr)
                ns.append(dst.numel())
                self._note_copy(p)
            elif g.is_cuda and g.dtype == b.dtype and _same_layout(g, p) and _is_dense(g):
                srcs.append(g)
                dptrs.append(dptr)
                ns.append(dst.numel())
                self._note_copy(p)
            else:
                dst.copy_(g)
                self._note_copy(p)
        if srcs:
            C = _ext.get(required=True)
            code = mt.DTYPE_CODE[b.dtype]
            C.mt_copy([g.data_ptr() for g in srcs], dptrs, ns, code, code, 1.0,
                      torch.cuda.current_stream(b.device).cuda_stream)
        # from here on p.grad aliases the (soon reduced) flat buffer, as in "view" mode
        for p, dst, _ in views:
            p.grad = dst

    def _grad_views(self, b: _Bucket) -> list:
        """``(param, view of its flat-gradient slice, slice address)`` per parameter (cached)."""
        v = self._views.get(b.index)
        if v is None:
            es = b.flat_grad.element_size()
            base = b.flat_grad.data_ptr()
            v = [(p, _strided_view(b.flat_grad, p, o), base + o * es) for p, o in zip(b.params, b.offsets)]
            self._views[b.index] = v
        return v

    def reduce_gradients(self):
        """Make sure every bucket has been allreduced (launch the rest, in order) and wait."""
        if self.overlap_opt:
            raise RuntimeError("DDP.reduce_gradients: with overlap_opt the updates run with the "
                               "reductions; call step() (or build the engine with overlap_opt=False)")
        for b in self.buckets:
            b.ready = True
        self._launch_ready()
        for b in self.buckets:
            self._pack(b)
            self._finish(b)

    def _fence_all(self):
        """One compute-stream fence for all buckets when the communicator runs every collective on
        one in-order stream (RcclComm): waiting for the last bucket's event covers the others. A
        cross-queue wait costs the compute queue a dependency round trip each (measured: the
        eager --force-comm step paid ~0.3 ms over 5 per-bucket waits, the captured graph none)."""
        if not getattr(self.comm, "in_order", False):
            return
        works = [b.work for b in self.buckets if b.work is not None]
        if len(works) < 2 or not all(hasattr(w, "covered") for w in works):
            return
        works[-1].wait()
        for w in works[:-1]:
            w.covered()

    def _finish(self, b: _Bucket):
        """Make the compute stream wait for bucket ``b``'s allreduce (and cast it back)."""
        if b.work is not None:
            b.work.wait()
            b.work = None
            if b.comm_buf is not None and self.comm_dtype != b.dtype:
                mt.unpack(b.comm_buf, [b.flat_grad], [0])

    def _arm_carry(self):
        """``step(zero_grad=False)`` with communication: the flat buffers hold the REDUCED sum
        S1. Accumulating the next backward into them and reducing again would apply
        ``W*S1 + S2``; the reference semantics (gradients summed over ranks, then applied:
        ``/root/reference/src/optimizer.jl:20-23``) ask for ``S1 + S2``. So S1 moves to a carry
        buffer that is added back after the next reduction, and the next forward (a one-shot
        pre-hook) clears the local gradients so only the new local part is reduced. Until that
        forward ``p.grad`` still shows S1."""
        for b in self.buckets:
            if b.carry is None:
                b.carry = torch.empty_like(b.flat_grad)
            b.carry.copy_(b.flat_grad)
        self._carry_live = True
        if self._carry_hook is None:
            self._carry_hook = self.module.register_forward_pre_hook(lambda m, a: self._start_carry())

    def _start_carry(self):
        """First forward after ``step(zero_grad=False)``: drop the (reduced) gradients."""
        if self._carry_hook is not None:
            self._carry_hook.remove()
            self._carry_hook = None
        if self.grad_mode == "view":
            mt.fill_([b.flat_grad for b in self.buckets], 0.0)
        else:
            for b in self.buckets:
                for p in b.params:
                    p.grad = None

    def _drop_carry(self):
        self._carry_live = False
        if self._carry_hook is not None:
            self._carry_hook.remove()
            self._carry_hook = None

    def _add_carry(self, b: _Bucket):
        if self._carry_live and b.carry is not None:
            b.flat_grad.add_(b.carry)

    def step(self, zero_grad: bool = True):
        """Finish the gradient allreduces and apply the fused optimiser to every bucket.

        The buckets are re-armed here whatever ``zero_grad`` is, so a following
        backward + ``step(zero_grad=False)`` (gradient accumulation across steps)
        launches, packs and waits on every bucket again; the applied gradient of that
        step is the sum over ranks of both backwards' gradients (see ``_arm_carry``).
        """
        gscale = 1.0 / self.world if self.average else 1.0
        if not (self.overlap_opt and self._masters_synced):
            self._sync_masters()
        if self._carry_hook is not None:
            self._start_carry()  # no forward since step(zero_grad=False): no new local gradient
        if self.overlap_opt:
            self._step_overlapped()
            self._finish_step(zero_grad)
            return
        if not self.communicate and self.grad_mode == "steal":
            # nothing to reduce: the optimiser reads autograd's gradients where they are
            for b in self.buckets:
                if not self._apply_direct(b, gscale):
                    self._pack(b)
                    self._apply(b, gscale)
            self._finish_step(zero_grad)
            return
        for b in self.buckets:
            if not b.launched:
                b.ready = True
        self._launch_ready()
        if self.timing and self.device.type == "cuda":
            # exposed communication: from the end of backward (all grads produced on the
            # compute stream) until the compute stream may consume the last reduced bucket
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self._fence_all()
            for b in self.buckets:
                self._pack(b)
                self._finish(b)
            e1.record()
            self._comm_events.append((e0, e1))
            for b in self.buckets:
                self._add_carry(b)
                self._apply(b, gscale)
        else:
            self._fence_all()
            for b in self.buckets:
                self._pack(b)
                self._finish(b)
                self._add_carry(b)
                self._apply(b, gscale)
        self._finish_step(zero_grad)

    def _step_overlapped(self):
        """step() with the per-bucket updates already enqueued during backward: enqueue the
        rest (buckets whose hooks did not complete them: unused parameters, no_sync), then ONE
        compute-stream fence on the optimiser stream (in order: it covers every bucket's
        allreduce and update)."""
        for b in self.buckets:
            if not b.launched:
                b.ready = True
        if self.timing and self.communicate:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        self._launch_ready()
        if self._opt_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
        for b in self.buckets:
            if b.work is not None:
                b.work.covered() if hasattr(b.work, "covered") else b.work.wait()
                b.work = None
        if self.timing and self.communicate:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._comm_events.append((e0, e1))

    def _finish_step(self, zero_grad: bool):
        if self.kind == "adam":
            fused.adam_advance_(self.hyper, self.adam.beta[0], self.adam.beta[1])
        self.step_count += 1
        if self.watchdog is not None:
            self.watchdog.check()
        if self.debug_checks and self.world > 1:
            check_replicas(self.module, comm=runtime.cpu_comm())
        self._rearm()
        self._record_versions()  # the optimiser's own writes are not "outside" changes
        if zero_grad:
            self.zero_grad()
        elif self.communicate:
            self._arm_carry()

    # ------------------------------------------------------------------ masters
    def _record_versions(self):
        self._versions = [[p._version for p in b.params] for b in self.buckets]

    def _sync_masters(self):
        """Pick up parameter changes made outside the engine (``load_state_dict``,
        ``checkpoint.load``, ``synchronize``, in-place edits): a changed version counter
        means the fp32 master of that parameter is stale, so it is re-read from the param."""
        for b, vs in zip(self.buckets, self._versions):
            for i, p in enumerate(b.params):
                if p._version != vs[i]:
                    if b.master is not None:
                        o = b.offsets[i]
                        with torch.no_grad():
                            _strided_view(b.master, p, o).copy_(p.detach())
                    vs[i] = p._version

    def refresh_master(self):
        """Re-read every fp32 master weight from its (low-precision) parameter."""
        with torch.no_grad():
            for b in self.buckets:
                if b.master is not None:
                    b.master.copy_(b.flat_param)
        self._record_versions()

    def exposed_comm_ms(self, reset: bool = True) -> float | None:
        """Mean exposed (not overlapped with backward) allreduce time per step, in ms,
        over the steps run with ``timing=True`` since the last reset; None if none."""
        if not self._comm_events:
            return None
        torch.cuda.synchronize(self.device)
        ms = [a.elapsed_time(b) for a, b in self._comm_events]
        if reset:
            self._comm_events.clear()
        return sum(ms) / len(ms)

    def _apply(self, b: _Bucket, gscale: float):
        masters = [b.master] if b.master is not None else None
        if self.kind == "adam":
            a = self.adam
            fused.adam_([b.flat_param], [b.flat_grad], [b.exp_avg], [b.exp_avg_sq], lr=a.eta, beta1=a.beta[0],
                        beta2=a.beta[1], eps=a.epsilon, bc1=0.0, bc2=0.0, weight_decay=self.wd,
                        grad_scale=gscale, masters=masters, dev_hyper=self.hyper)
        else:
            mom = {"descent": 0.0}.get(self.kind, getattr(self.rule, "rho", 0.0))
            fused.sgd_([b.flat_param], [b.flat_grad], [b.exp_avg] if b.exp_avg is not None else None,
                       lr=self.rule.eta, momentum=mom, nesterov=self.kind == "nesterov", weight_decay=self.wd,
                       grad_scale=gscale, masters=masters, dev_lr=self.hyper)

    def _apply_direct(self, b: _Bucket, gscale: float) -> bool:
        """Fused optimiser on the autograd gradients in place (no pack). False if some gradient
        cannot be read directly (missing, other dtype/layout/device): the caller packs instead."""
        grads = []
        for p in b.params:
            g = p.grad
            if g is None:
                return False
            if not (g.dtype is b.dtype and g.stride() == p.stride() and g.device == b.device):
                if g.dtype != b.dtype or g.device != b.device or not _same_layout(g, p) or not _is_dense(g):
                    return False
            grads.append(g)
        st = self._direct_cache.get(b.index)
        if st is None:
            def sl(flat):
                return [flat[o:o + p.numel()] for p, o in zip(b.params, b.offsets)] if flat is not None else None
            st = (sl(b.flat_param), sl(b.exp_avg), sl(b.exp_avg_sq), sl(b.master))
            self._direct_cache[b.index] = st
        ps, ms, vs, ws = st
        # the flat slices are in memory order; a gradient with its parameter's strides is too
        gs = [g.view(-1) if g.is_contiguous() else g.as_strided((g.numel(),), (1,)) for g in grads]
        if self.kind == "adam":
            a = self.adam
            fused.adam_(ps, gs, ms, vs, lr=a.eta, beta1=a.beta[0], beta2=a.beta[1], eps=a.epsilon, bc1=0.0,
                        bc2=0.0, weight_decay=self.wd, grad_scale=gscale, masters=ws, dev_hyper=self.hyper)
        else:
            mom = {"descent": 0.0}.get(self.kind, getattr(self.rule, "rho", 0.0))
            fused.sgd_(ps, gs, ms, lr=self.rule.eta, momentum=mom, nesterov=self.kind == "nesterov",
                       weight_decay=self.wd, grad_scale=gscale, masters=ws, dev_lr=self.hyper)
        return True

    def set_lr(self, lr: float):
        """Change the learning rate (device-side, so captured graphs see it)."""
        self.hyper[0].fill_(lr)
        if self.kind == "adam":
            self.adam.eta = lr
        else:
            self.rule.eta = lr

    # ------------------------------------------------------------------ state
    def optimiser_state(self):
        """Optimisers.jl-layout state tree ``{name: Leaf(rule, state)}`` (views, no copies)."""
        out = {}
        if self.kind == "adam":
            bt = self.hyper[1:].tolist()
        for b in self.buckets:
            for name, p, o in zip(b.names, b.params, b.offsets):
                n = p.numel()
                # moments follow the parameter's memory order (NHWC for channels_last weights)
                if self.kind == "adam":
                    st = (_strided_view(b.exp_avg, p, o), _strided_view(b.exp_avg_sq, p, o), tuple(bt))
                elif b.exp_avg is not None:
                    st = _strided_view(b.exp_avg, p, o)
                else:
                    st = None
                out[name] = O.Leaf(self.rule, st)
        return out

    def state_dict(self):
        return {
            "module": self.module.state_dict(),
            "step": self.step_count,
            "hyper": self.hyper.detach().cpu(),
            "buckets": [{"master": b.master.detach().cpu() if b.master is not None else None,
                         "m": b.exp_avg.detach().cpu() if b.exp_avg is not None else None,
                         "v": b.exp_avg_sq.detach().cpu() if b.exp_avg_sq is not None else None}
                        for b in self.buckets],
        }

    def load_state_dict(self, sd):
        with torch.no_grad():
            self.module.load_state_dict(sd["module"])
            self.step_count = int(sd["step"])
            self.hyper.copy_(sd["hyper"])
            for b, s in zip(self.buckets, sd["buckets"]):
                if b.master is not None:
                    if s["master"] is not None:
                        b.master.copy_(s["master"])
                    else:  # checkpoint without masters: start them from the loaded params
                        b.master.copy_(b.flat_param)
                if s["m"] is not None:
                    b.exp_avg.copy_(s["m"])
                if s["v"] is not None:
                    b.exp_avg_sq.copy_(s["v"])
        self._record_versions()

    def num_parameters(self) -> int:
        return sum(p.numel() for b in self.buckets for p in b.params)

    def comm_summary(self) -> dict:
        """What the engine communicates per step (for bench records)."""
        return {"communicate": self.communicate, "force_comm": self.force_comm,
                "overlap": bool(self.overlap and self.communicate), "grad_mode": self.grad_mode,
                "buckets": len(self.buckets),
                "bucket_mb": [round(b.numel * b.flat_grad.element_size() / 2 ** 20, 2) for b in self.buckets],
                "comm": (self.comm.name if self.communicate else "none"),
                "direct_grads": self.direct_grads, "overlap_opt": self.overlap_opt,
                "bucket_plan": self.bucket_plan,
                "comm_probe": self.comm_probe,
                # gradients the packs copied per step so far (0: every one delivered in place)
                "pack_copies_per_step": round(self.pack_copies / max(1, self.step_count), 2),
                # the parameter shapes the packs copied (total over the steps so far), most first
                "pack_copied_shapes": dict(sorted(self.pack_copied.items(), key=lambda kv: -kv[1])[:8])}

    def bucket_summary(self) -> list:
        return [{"index": b.index, "dtype": str(b.dtype), "numel": b.numel, "params": len(b.params),
                 "mbytes": b.numel * b.flat_grad.element_size() / 2 ** 20} for b in self.buckets]

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


__all__ = ["DDP"]
