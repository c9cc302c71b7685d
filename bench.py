#!/usr/bin/env python
"""North-star benchmark: ResNet-50 data-parallel training throughput (images/s).

``python bench.py --gpus N --steps K --warmup W`` — for N > 1 launched by the
driver as ``torch.distributed.run --nproc-per-node N`` (one rank per GPU,
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the environment).

Workload (BASELINE.json: "images/sec ResNet50 Lux.jl DDP at 1/2/4/8 MI355X"):
ResNet-50 (25.6 M params, torchvision v1.5 layout), bf16 compute with fp32
master weights + fp32 Adam moments (BatchNorm parameters fp32), channels_last,
synthetic ImageNet batches (224x224x3, 1000 classes, random-init weights),
per-GPU batch fixed as N grows (weak scaling). Every timed step runs the full
forward, cross-entropy loss, backward with bucketed RCCL allreduce overlapped
on a side stream (N > 1), and the fused HIP Adam update of every parameter.

Timing: W untimed warmup steps, barrier + device sync, K timed steps, barrier
+ device sync; the max elapsed time over ranks is reported. Rank 0 prints one
JSON line; ``value`` is the whole-job images/s.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

METRIC = "images/sec ResNet50 Lux.jl DDP at 1/2/4/8 MI355X; scaling efficiency"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", "256")), help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--image", type=int, default=None, help="input resolution (default: 224; DEQ: 28, MNIST-shaped)")
    ap.add_argument("--conv", default=os.environ.get("BENCH_CONV", "hybrid"), choices=["gemm", "miopen", "fused", "hybrid"])
    ap.add_argument("--norm", default=os.environ.get("BENCH_NORM", "fused"), choices=["torch", "fused"])
    ap.add_argument("--optimizer", default="adam", choices=["adam", "momentum"])
    ap.add_argument("--memory-format", default=os.environ.get("BENCH_MEMFMT", "auto"),
                    choices=["auto", "channels_last", "contiguous"],
                    help="activation layout (auto: the model's `memory_format` attribute, else channels_last)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--force-comm", action="store_true",
                    help="issue the gradient collectives even at N=1 (hooks, packing, RCCL on the comm "
                         "stream): measures the data-parallel layer's own cost on one GPU")
    ap.add_argument("--emulate-comm", default="",
                    help="WGS:GBPS — with --force-comm at N=1, hold WGS workgroups on the comm stream for the "
                         "time an 8-rank ring allreduce of each bucket takes at GBPS (RCCL's CU footprint)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on cuda:0 with gloo collectives on device tensors (RCCL refuses a "
                         "shared GPU): runs the N>1 code path on a 1-GPU box; no throughput claim")
    ap.add_argument("--graph", action="store_true", help="capture the step in a HIP graph")
    ap.add_argument("--deq-solver", default="",
                    help="DEQ models: solver settings as k=v pairs, e.g. 'tol=1e-2,bwd_tol=1e-2,max_iter=30'")
    ap.add_argument("--overlap-opt", type=int, default=None, choices=[0, 1],
                    help="per-bucket optimiser overlap: each bucket's fused update is enqueued during "
                         "backward behind its allreduce (default: on when the step communicates — N>1 or "
                         "--force-comm — and not --graph; the bench loop is backward -> step())")
    ap.add_argument("--api", default="ddp", choices=["ddp", "functional"],
                    help="ddp: the DDP engine (hooks, buckets born in the comm buffers, fused optimiser); "
                         "functional: the reference's API shape (src/optimizer.jl:45-65) — the nested "
                         "parameter tree's gradients through allreduce_gradients(like=ps), then "
                         "Optimisers.update! (fused multi-tensor kernels)")
    ap.add_argument("--miopen-find", type=int, default=int(os.environ.get("BENCH_MIOPEN_FIND", "1")))
    ap.add_argument("--choices", default=os.environ.get("BENCH_CHOICES", "measure"), choices=["measure", "shipped"],
                    help="measure (default): per-shape kernel choices (ours vs MIOpen, tile configs) timed at the "
                         "first step; shipped: read tuning/kernel_choices/<model>_bs<batch>.jsonl (no first-step "
                         "timing, no run-to-run flips; measured 0.8%% slower than a fresh measurement on one box, "
                         "profiles/r4i_bench_choices_ab.jsonl)")
    ap.add_argument("--dump-choices", default="", help="write the per-shape kernel choices in use to this file")
    ap.add_argument("--tunableop", default=os.environ.get("BENCH_TUNABLEOP", "auto"), choices=["auto", "off"],
                    help="auto: use the shipped hipBLASLt/rocBLAS GEMM selections (tuning/tunableop/<model>.csv)")
    return ap.parse_args()


def _gelu_form() -> str:
    from fluxmpi_amd.ops import gelu as GL

    return GL.FORM


class Functional:
    """The reference's functional training step as a DDP stand-in for the bench loop: the model's
    parameters as a nested tree (module path -> leaf), broadcast from rank 0 (``synchronize``), the
    gradient tree reduced by ``allreduce_gradients(gs, like=ps)`` (averaged, as the DDP engine's
    ``average=True``; ``like``: a rank without some gradient still joins every bucket) and applied
    by ``Optimisers.update!`` (one fused multi-tensor launch per dtype group)."""

    def __init__(self, FluxMPI, O, model, rule):
        from fluxmpi_amd.parallel.bucket import plan_buckets
        from fluxmpi_amd.parallel.comm import ReduceOp

        self.F, self.O, self.module = FluxMPI, O, model
        self.op = ReduceOp.AVG
        self.ps: dict = {}
        for name, p in model.named_parameters():
            d = self.ps
            *path, leaf = name.split(".")
            for k in path:
                d = d.setdefault(k, {})
            d[leaf] = p
        FluxMPI.synchronize(model, root_rank=0)  # parameters and buffers (BatchNorm statistics)
        # the optimiser updates fp32 parameters (as a Lux / Optimisers.jl user keeps Float32
        # parameters: Optimisers.jl casts beta to eltype(x), and BFloat16(0.999) == 1 would make
        # Adam's bias correction 0/0); the bf16 compute copies are refreshed from them by one
        # multi-tensor cast launch per step
        self.params = [p for p in model.parameters()]
        self.ps32 = self._map(self.ps, lambda p: p.detach().float() if p.dtype != torch.float32 else p)
        self.low = [(p, q) for p, q in zip(self._leaves(self.ps), self._leaves(self.ps32)) if q is not p]
        self.st = O.setup(rule, self.ps32)
        self.plan = plan_buckets([p.detach() for p in self.params if p.requires_grad], None)
        self.communicate = FluxMPI.total_workers() > 1 or os.environ.get("FLUXMPI_FORCE_COMM") == "1"
        self.timing = False
        self.step_count = 0

    @classmethod
    def _map(cls, t, fn):
        return {k: cls._map(v, fn) for k, v in t.items()} if isinstance(t, dict) else fn(t)

    @classmethod
    def _leaves(cls, t):
        return [x for v in t.values() for x in cls._leaves(v)] if isinstance(t, dict) else [t]

    def __call__(self, x):
        return self.module(x)

    def _grads(self, t):
        return {k: self._grads(v) for k, v in t.items()} if isinstance(t, dict) else t.grad

    def step(self):
        gs = self.F.allreduce_gradients(self._grads(self.ps), op=self.op, like=self.ps)
        self.O.update_(self.st, self.ps32, gs)
        if self.low:  # the compute copies from the updated fp32 parameters, one launch per dtype
            from fluxmpi_amd.ops import _ext
            from fluxmpi_amd.ops.multi_tensor import DTYPE_CODE
            groups: dict = {}
            for p, q in self.low:
                groups.setdefault(p.dtype, []).append((p, q))
            for dt, pq in groups.items():
                if not pq[0][0].is_cuda:
                    for p, q in pq:
                        p.data.copy_(q)
                    continue
                C = _ext.get(required=True)
                C.mt_copy([q.data_ptr() for _, q in pq], [p.data_ptr() for p, _ in pq], [p.numel() for p, _ in pq],
                          DTYPE_CODE[torch.float32], DTYPE_CODE[dt], 1.0,
                          torch.cuda.current_stream(pq[0][0].device).cuda_stream)
        for p in self.params:
            p.grad = None
        self.step_count += 1

    def exposed_comm_ms(self):
        return None

    def comm_summary(self) -> dict:
        mb = [round(t[5] * t[2].itemsize / 2 ** 20, 2) for t in self.plan]  # packed buckets and direct leaves
        return {"api": "functional", "communicate": self.communicate, "overlap": False,
                "buckets": len(self.plan), "bucket_mb": mb,
                "comm": self.F.backend_name() if self.communicate else "none"}


def selfcheck_or_code(FluxMPI, world: int, rank: int, dev):
    """The device communicator's own report (RCCL: ncclCommCount / UserRank / CuDevice, stream
    priority) checked against WORLD_SIZE / RANK / the pinned device: the dict on success, exit
    code 4 on a mismatch (no number is reported from a communicator that is not what it claims)."""
    from fluxmpi_amd.parallel import runtime
    from fluxmpi_amd.parallel.selfcheck import CommSelfCheckError, comm_selfcheck

    rep, ok = {}, 1
    try:
        rep = comm_selfcheck(runtime.device_comm(), world, rank, getattr(dev, "index", None))
    except CommSelfCheckError as e:
        print(f"bench.py: rank {rank}: communicator self-check failed: {e}", file=sys.stderr, flush=True)
        ok = 0
    if world > 1:  # every rank leaves together (a lone failing rank would hang the others' collectives)
        ok = int(FluxMPI.allreduce(torch.tensor([ok], dtype=torch.int64), min).item())
    return rep if ok else 4


def comm_env() -> dict:
    """The RCCL / NCCL tuning environment of this run (channel counts, protocols, algorithms,
    P2P and xGMI settings): recorded beside the number so a scaling run states what it ran with.
    Nothing is set by this bench; RCCL picks channels and protocols itself when these are unset."""
    keys = sorted(k for k in os.environ if k.startswith(("NCCL_", "RCCL_")))
    return {k: os.environ[k] for k in keys}


def main():
    args = parse()
    if args.image is None:
        args.image = {"deq": 28, "deq_cifar": 32}.get(args.model, 224)
    if args.api == "functional" and args.force_comm:
        os.environ["FLUXMPI_FORCE_COMM"] = "1"  # allreduce_gradients communicates even at N=1
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models import build_model
    from fluxmpi_amd.parallel.ddp import DDP

    # PyTorch TunableOp: per-shape GEMM solution choices recorded on MI355X (read-only here)
    tuned = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "tunableop", f"{args.model}.csv")
    use_tunableop = args.tunableop == "auto" and os.path.exists(tuned) and "PYTORCH_TUNABLEOP_ENABLED" not in os.environ
    if use_tunableop:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.record_untuned_enable(False) if hasattr(torch.cuda.tunable, "record_untuned_enable") else None
        torch.cuda.tunable.read_file(tuned)
        # results are written back at exit: keep that copy out of the repository
        torch.cuda.tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                     f"fluxmpi_tunableop_{os.getuid()}_{args.model}.csv"))
    if args.emulate_comm:
        os.environ["FLUXMPI_EMULATE_COMM"] = args.emulate_comm
    if args.same_device:
        os.environ["FLUXMPI_BACKEND"] = "gloo-device"
        FluxMPI.Init(gpu_devices=[0] * int(os.environ.get("WORLD_SIZE", "1")))
    else:
        FluxMPI.Init()
    # MIOpen find mode, seeded with the tuning db recorded on MI355X (tuning/miopen): the
    # per-shape solver choice without the ~3.5 min search. --miopen-find 0: immediate mode.
    if args.miopen_find:
        from fluxmpi_amd.utils.miopen import install_tuned_db

        install_tuned_db(rank=int(os.environ.get("LOCAL_RANK", "0")))
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    # shipped per-shape kernel choices (recorded on MI355X; the analogue of the MIOpen find-db):
    # no first-step measurement, no run-to-run flips of shapes where both kernels are within noise
    choices = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "kernel_choices",
                           f"{args.model}_bs{args.batch}.jsonl")
    use_choices = args.choices == "shipped" and os.path.exists(choices) and "FLUXMPI_KERNEL_CHOICES" not in os.environ
    if use_choices:
        from fluxmpi_amd.ops import fused_block

        fused_block.load_choices(choices)
    rank, world = FluxMPI.local_rank(), FluxMPI.total_workers()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but world size {world}", file=sys.stderr)
    dev = FluxMPI.device()
    if dev.type != "cuda":
        print("bench.py needs a GPU", file=sys.stderr)
        return 2

    torch.manual_seed(1234 + rank)
    solver = {}
    for kv in filter(None, args.deq_solver.split(",")):
        k, v = kv.split("=")
        solver[k.strip()] = int(v) if k.strip() in ("max_iter", "bwd_iter", "check_lag", "m", "bwd_m", "skip", "restart", "skip_detach") else float(v)
    model = build_model(args.model, conv_impl=args.conv, norm=args.norm, **solver)
    memfmt = {"channels_last": torch.channels_last, "contiguous": torch.contiguous_format}.get(
        args.memory_format, getattr(model, "memory_format", torch.channels_last))
    model = model.to(dev, memory_format=memfmt)
    # bf16 compute; BatchNorm affine params + running stats stay fp32
    for m in model.modules():
        is_norm = isinstance(m, torch.nn.modules.batchnorm._BatchNorm) or type(m).__name__ == "FusedBatchNorm2d"
        if not is_norm:
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    if world > 1 and not args.same_device and FluxMPI.backend_name() != "rccl":
        # no silent fallback: an N>1 number must come from the native RCCL communicator
        print(f"bench.py: device backend is {FluxMPI.backend_name()!r}, not the native 'rccl' "
              "communicator; refusing to report an N>1 number (use --same-device for a rehearsal)",
              file=sys.stderr)
        return 3
    comm_report = selfcheck_or_code(FluxMPI, world, rank, dev)
    if isinstance(comm_report, int):
        return comm_report
    rule = O.Adam(1e-3) if args.optimizer == "adam" else O.Momentum(0.1, 0.9)
    if args.api == "functional":
        if args.graph:
            print("bench.py: --graph needs --api ddp", file=sys.stderr)
            return 2
        ddp = Functional(FluxMPI, O, model, rule)
    else:
        ovo = args.overlap_opt
        if ovo is None:  # the engine's contract (every backward followed by step()) holds here
            ovo = int((world > 1 or args.force_comm) and not args.graph and not args.no_overlap)
        ddp = DDP(model, rule, average=True, overlap=not args.no_overlap, force_comm=args.force_comm,
                  overlap_opt=bool(ovo))

    B = args.batch
    gx = torch.Generator(device=dev).manual_seed(rank)
    # DEQs: MNIST-shaped (deq) and CIFAR-shaped (deq_cifar), the FastDEQ examples' data
    cin, ncls = {"deq": (1, 10), "deq_cifar": (3, 10)}.get(args.model, (3, 1000))
    x = torch.randn(B, cin, args.image, args.image, device=dev, generator=gx).to(torch.bfloat16)
    x = x.contiguous(memory_format=memfmt)
    y = torch.randint(0, ncls, (B,), device=dev, generator=gx)

    deq = getattr(model, "deq", None)  # DEQ: solver iterations per step are reported with the rate
    iters: list = []

    def step():
        out = ddp(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        ddp.step()
        if deq is not None:
            iters.append((deq.last_iters, deq.last_bwd_iters, deq.last_res))
        return loss

    calibrated = False
    if world > 1 and args.api == "ddp":
        # per-shape kernel choices measured once on rank 0 with no collective in flight, shared
        # with every rank and frozen (parallel/autotune.py): all ranks run the same kernels
        from fluxmpi_amd.parallel.autotune import calibrate

        calibrate(ddp, lambda: F.cross_entropy(ddp(x).float(), y).backward())
        calibrated = True

    if args.graph and args.model == "deq":
        # the implicit layer's solver lengths are data dependent (host-side loop exits), which a
        # captured graph cannot express; the lagged device-side checks remove the queue drains instead
        print("bench.py: --graph is not supported for the DEQ model (data-dependent solver loops)", file=sys.stderr)
        return 2
    if args.graph:
        from fluxmpi_amd.parallel.graph import GraphedStep

        graphed = GraphedStep(ddp, lambda d, xx, yy: F.cross_entropy(d(xx).float(), yy), x, y)
        step = lambda: graphed(x, y)  # noqa: E731

    for _ in range(args.warmup):
        step()
    iters.clear()
    FluxMPI.barrier()
    torch.cuda.synchronize()
    from fluxmpi_amd.models import deq as _deq_mod
    wait0 = _deq_mod.HOST_WAIT_S
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    t_host = time.perf_counter() - t0  # the host's enqueue time: ~wall when launch-bound
    t_wait = _deq_mod.HOST_WAIT_S - wait0  # DEQ: blocked on the solvers' convergence flags
    timed_iters = list(iters[:args.steps])
    torch.cuda.synchronize()
    FluxMPI.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        per_rank = [float(v) for v in FluxMPI.allgather(torch.tensor([dt], dtype=torch.float64)).flatten()]
    else:
        per_rank = [dt]
    dt_max = max(per_rank)
    lval = float(loss.item())
    exposed = None
    if ddp.communicate and not args.graph and args.api == "ddp":
        # after the timed region: a few steps with event timing around the gradient-allreduce
        # wait (exposed = not hidden behind backward), max over ranks
        ddp.timing = True
        for _ in range(3):
            step()
        ddp.timing = False
        e = ddp.exposed_comm_ms()
        exposed = e or 0.0
        if world > 1:
            exposed = FluxMPI.allreduce(torch.tensor([exposed], dtype=torch.float64), max).item()
    if args.dump_choices and rank == 0:
        from fluxmpi_amd.ops import fused_block

        with open(args.dump_choices, "w") as f:
            f.write("\n".join(fused_block.dump_choices()) + "\n")
    cs = ddp.comm_summary()
    if rank == 0:
        ips = world * B * args.steps / dt_max
        names = {"resnet50": "ResNet50", "vit_b16": "ViT-B/16", "deq": "DEQ", "deq_cifar": "DEQ-CIFAR (FastDEQ width)"}
        mname = names.get(args.model, args.model)
        metric = METRIC if args.model == "resnet50" else METRIC.replace("ResNet50 Lux.jl", f"{mname}")
        rec = {
            "metric": metric, "value": round(ips, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt_max / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": mname, "global_batch": world * B, "per_gpu_batch": B, "seq_len": None,
                       "image_size": args.image, "parallelism": f"dp{world}", "optimizer": args.optimizer,
                       "conv": args.conv, "norm": args.norm, "memory_format": "contiguous" if memfmt is torch.contiguous_format else "channels_last", "backend": FluxMPI.backend_name(),
                       "miopen_find": bool(args.miopen_find), "hip_graph": bool(args.graph),
                       "tunableop": use_tunableop,
                       "kernel_choices": ("shipped" if use_choices else "measured")
                       + ("+rank0-calibrated" if calibrated else ""),
                       "host_ms_per_step": round(1000 * t_host / args.steps, 3),
                       # DEQ: the host's time net of its waits on the solvers' convergence flags
                       # (those waits are the data-dependent control flow, not host work)
                       **({"host_flag_wait_ms_per_step": round(1000 * t_wait / args.steps, 3),
                           "host_busy_ms_per_step": round(1000 * (t_host - t_wait) / args.steps, 3)}
                          if t_wait > 0 else {}),
                       "loss": round(lval, 4), "loss_finite": math.isfinite(lval),
                       # what the data-parallel layer actually did: at N=1 nothing is communicated
                       # (overlap false, comm "none") unless --force-comm
                       **cs, "exposed_comm_ms": None if exposed is None else round(exposed, 3),
                       **({"emulate_comm": args.emulate_comm} if args.emulate_comm else {}),
                       "grid_rounds": int(os.environ.get("FLUXMPI_GRID_ROUNDS", "1")),
                       # the communicator's own report (checked against the launch before timing)
                       # and the per-rank spread of the timed region
                       **comm_report, "comm_env": comm_env(),
                       "rank_ms_per_step_min": round(1000 * min(per_rank) / args.steps, 3),
                       "rank_ms_per_step_max": round(1000 * max(per_rank) / args.steps, 3),
                       **({"gelu": _gelu_form()} if args.model == "vit_b16" else {}),
                       **({"deq_solver": {**{k: getattr(deq, k) for k in ("max_iter", "tol", "bwd_iter", "bwd_tol", "m", "bwd_m", "beta", "lam", "restart")},
                                          "skip": deq.skip is not None}}
                          if deq is not None else {}),
                       **({"deq_fwd_iters_per_step": round(sum(i[0] for i in timed_iters) / len(timed_iters), 2),
                           "deq_bwd_iters_per_step": round(sum(i[1] for i in timed_iters) / len(timed_iters), 2),
                           "deq_fwd_residual_max": max([float(i[2]) for i in timed_iters if i[2] is not None],
                                                       default=None)}
                          if timed_iters else {})},
        }
        print(json.dumps(rec), flush=True)
    FluxMPI.Finalize()
    if not math.isfinite(lval):
        # a non-finite loss means a kernel produced garbage: NaN/Inf data also changes the timing
        # (lower power draw, higher clocks), so the number above is not a valid measurement
        print(f"bench.py: non-finite loss {lval} - the measurement is invalid", file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
