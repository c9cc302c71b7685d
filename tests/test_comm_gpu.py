"""The device collective path on one MI355X.

A 1-GPU box cannot host an N>1 RCCL communicator (RCCL refuses a duplicate
device: ``profiles/r2_probe_rccl_two_ranks_one_gpu.json``), so these tests
drive every piece of the N>1 device path that can run there:

* ``force_comm``: the DDP engine at world 1 registers its hooks, packs, and
  issues real ``ncclAllReduce`` calls on the communicator's priority stream
  with event fencing; the parameters must be bitwise equal to the no-comm run
  (a SUM over one rank is the identity);
* HIP-graph capture of those RCCL calls, the watchdog tracking real stream
  works, bool reductions, send/recv (alltoall), abort;
* the host-staged path behind ``disable_cudampi_support`` in a fresh process;
* two ranks sharing ``cuda:0`` through gloo on device tensors (the
  ``gloo-device`` backend): DDP with hook-driven overlap against the
  summed-gradient single-process reference (``tests/test_ddp.py`` on CPU).
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _init():
    import fluxmpi_amd as FluxMPI

    FluxMPI.Init()
    assert FluxMPI.backend_name() == "rccl", FluxMPI.backend_name()
    return FluxMPI


def _mlp(seed, dtype=torch.float32):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(32, 256), torch.nn.Tanh(), torch.nn.Linear(256, 256), torch.nn.Tanh(),
                               torch.nn.Linear(256, 8)).to("cuda", dtype)


def _data(dtype=torch.float32):
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(64, 32, device="cuda", generator=g).to(dtype)
    return x, torch.randn(64, 8, device="cuda", generator=g).to(dtype)


@pytest.mark.parametrize("grad_mode", ["steal", "view"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_force_comm_bitwise_equal(gpu_ext, grad_mode, dtype):
    _init()
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.comm import RcclComm
    from fluxmpi_amd.parallel.ddp import DDP

    m1, m2 = _mlp(0, dtype), _mlp(0, dtype)
    kw = dict(bucket_mb=0.1, first_bucket_mb=0.05, grad_mode=grad_mode)
    d1 = DDP(m1, O.Adam(1e-3), force_comm=True, **kw)
    d2 = DDP(m2, O.Adam(1e-3), **kw)
    assert isinstance(d1.comm, RcclComm) and d1.communicate and len(d1.buckets) >= 3
    assert not d2.communicate
    x, y = _data(dtype)
    for _ in range(4):
        for d in (d1, d2):
            F.mse_loss(d(x).float(), y.float()).backward()
        # the hooks launched every bucket's allreduce during backward, on the comm stream
        assert all(b.launched and b.work is not None for b in d1.buckets)
        d1.step()
        d2.step()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p, q)


def test_rccl_self_report(gpu_ext):
    """The native communicator reports itself (ncclCommCount / ncclCommUserRank / ncclCommCuDevice):
    what bench.py checks against WORLD_SIZE / RANK / the pinned device before timing."""
    _init()
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel import runtime
    from fluxmpi_amd.parallel.comm import RcclComm
    from fluxmpi_amd.parallel.selfcheck import CommSelfCheckError, comm_selfcheck

    c = runtime.device_comm()
    assert isinstance(c, RcclComm)
    rep = c.self_report()
    assert rep["rccl_nranks"] == FluxMPI.total_workers() == 1
    assert rep["rccl_rank"] == 0 and rep["rccl_device"] == FluxMPI.device().index
    assert rep["comm_priority"] == c.priority and rep["rccl_version"] > 0
    assert comm_selfcheck(c, 1, 0, FluxMPI.device().index) == rep
    with pytest.raises(CommSelfCheckError):
        comm_selfcheck(c, 2, 0, FluxMPI.device().index)


def test_force_comm_bench_construction(gpu_ext):
    """bench.py's DDP construction at N>1: parameter + buffer broadcast (fp32 BN stats, int64
    step counters that the pack kernels cannot move) and a step, over real RCCL calls."""
    _init()
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.parallel.ddp import DDP

    def build():
        torch.manual_seed(11)
        m = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused").to("cuda", memory_format=torch.channels_last)
        for mod in m.modules():
            if not (isinstance(mod, torch.nn.modules.batchnorm._BatchNorm) or type(mod).__name__ == "FusedBatchNorm2d"):
                for p in mod.parameters(recurse=False):
                    p.data = p.data.to(torch.bfloat16)
        return m

    m1, m2 = build(), build()
    assert any(b.dtype == torch.int64 for b in m1.buffers())
    d1 = DDP(m1, O.Adam(1e-3), average=True, force_comm=True)
    d2 = DDP(m2, O.Adam(1e-3), average=True)
    x = torch.randn(8, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    for d in (d1, d2):
        F.cross_entropy(d(x).float(), y).backward()
        d.step()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=4e-3)  # 2 bf16 ulps at |w| < 0.5


def test_force_comm_bf16_wire(gpu_ext):
    """fp32 gradients sent as bf16 (K5 cast kernels around a real RCCL call)."""
    _init()
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    m1, m2 = _mlp(1), _mlp(1)
    d1 = DDP(m1, O.Descent(0.05), force_comm=True, comm_dtype=torch.bfloat16, bucket_mb=0.1, first_bucket_mb=0.05)
    d2 = DDP(m2, O.Descent(0.05), bucket_mb=0.1, first_bucket_mb=0.05)
    x, y = _data()
    F.mse_loss(d1(x), y).backward()
    F.mse_loss(d2(x), y).backward()
    # the reduced gradient is the bf16 rounding of the local one
    d1.reduce_gradients()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.grad, q.grad.bfloat16().float(), rtol=0, atol=0)
    d1.step()
    d2.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-2, atol=1e-4)


def test_force_comm_graph_capture(gpu_ext):
    """The whole step, RCCL allreduces included, captured in one HIP graph and replayed."""
    _init()
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.parallel.graph import GraphedStep

    m1, m2 = _mlp(2, torch.bfloat16), _mlp(2, torch.bfloat16)
    d1 = DDP(m1, O.Adam(1e-3), force_comm=True, bucket_mb=0.1, first_bucket_mb=0.05)
    d2 = DDP(m2, O.Adam(1e-3), force_comm=True, bucket_mb=0.1, first_bucket_mb=0.05)
    assert d1.watchdog is not None
    x, y = _data(torch.bfloat16)

    def loss_fn(d, xx, yy):
        return F.mse_loss(d(xx).float(), yy.float())

    g = GraphedStep(d1, loss_fn, x, y, warmup=2)
    for _ in range(2):
        loss_fn(d2, x, y).backward()
        d2.step()
    for _ in range(3):
        g(x, y)
        loss_fn(d2, x, y).backward()
        d2.step()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p, q)
    assert d1.watchdog.error is None and not d1.watchdog._paused


def test_watchdog_tracks_real_stream_works(gpu_ext):
    _init()
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.comm import _StreamWork
    from fluxmpi_amd.parallel.ddp import DDP

    m = _mlp(3)
    d = DDP(m, O.Descent(0.01), force_comm=True, bucket_mb=0.1, first_bucket_mb=0.05)
    wd = d.watchdog
    wd.interval_s = 0.02
    x, y = _data()
    F.mse_loss(d(x), y).backward()
    works = [b.work for b in d.buckets]
    assert all(isinstance(w, _StreamWork) for w in works)
    assert len(wd._inflight) == len(d.buckets)
    d.step()
    torch.cuda.synchronize()
    for _ in range(200):
        if not wd._inflight:
            break
        time.sleep(0.02)
    assert not wd._inflight and wd.error is None


def test_rccl_bool_alltoall_abort(gpu_ext):
    from fluxmpi_amd.parallel.comm import CommAbortedError, RcclComm

    c = RcclComm(0, 1, torch.device("cuda", 0))
    b = torch.tensor([True, False, True, True], device="cuda")
    for op in ("+", "*", "max", "min"):
        t = b.clone()
        c.allreduce(t, op)
        torch.cuda.synchronize()
        assert t.dtype == torch.bool and torch.equal(t, b) and int(t.view(torch.uint8).max()) <= 1
    src = torch.arange(64, dtype=torch.float32, device="cuda")
    dst = torch.zeros_like(src)
    c.alltoall(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    c.abort("test")
    assert c.aborted and c._h.aborted
    with pytest.raises(CommAbortedError):
        c.allreduce(torch.ones(4, device="cuda"))
    c.check_async_error()  # an aborted communicator is no longer polled
    c.destroy()


def test_host_staged_preference_fresh_process(gpu_ext, tmp_path):
    """disable_cudampi_support() -> a NEW process runs the host-staged path (reference
    src/FluxMPI.jl:51-56, staging src/mpi_extensions.jl:97-155); results match RCCL."""
    prefs = tmp_path / "LocalPreferences.toml"
    env = dict(os.environ, FLUXMPI_PREFS=str(prefs), PYTHONPATH=ROOT)
    setp = "import fluxmpi_amd as F; F.disable_cudampi_support(True)"
    subprocess.run([sys.executable, "-c", setp], env=env, check=True, timeout=120)
    body = textwrap.dedent("""
        import torch, fluxmpi_amd as FluxMPI
        from fluxmpi_amd import optimisers as O
        from fluxmpi_amd.parallel.comm import HostStagedComm, RcclComm
        from fluxmpi_amd.parallel.ddp import DDP
        FluxMPI.Init()
        assert FluxMPI.backend_name() == "host-staged", FluxMPI.backend_name()
        from fluxmpi_amd.parallel import runtime
        assert isinstance(runtime.device_comm(), HostStagedComm)
        rc = RcclComm(0, 1, torch.device("cuda", 0))
        x = torch.randn(1000, device="cuda")
        a, b = x.clone(), x.clone()
        FluxMPI.allreduce(a, "+"); rc.allreduce(b)
        FluxMPI.bcast(a, 0); FluxMPI.reduce(a, "max", 0)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        torch.manual_seed(0)
        m = torch.nn.Linear(16, 4).cuda()
        d = DDP(m, O.Descent(0.1), force_comm=True)
        assert isinstance(d.comm, HostStagedComm)
        m(torch.randn(8, 16, device="cuda")).square().mean().backward()
        d.step(); torch.cuda.synchronize()
        rc.destroy(); FluxMPI.Finalize()
        print("HOST_STAGED_OK")
    """)
    r = subprocess.run([sys.executable, "-c", body], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "HOST_STAGED_OK" in r.stdout, r.stdout + r.stderr
    # without the preference the same program sees RCCL
    env2 = dict(env, FLUXMPI_PREFS=str(tmp_path / "none.toml"))
    r = subprocess.run([sys.executable, "-c", "import fluxmpi_amd as F; F.Init(); print(F.backend_name())"],
                       env=env2, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == "rccl", r.stdout + r.stderr


def worker_two_ranks_one_gpu():
    """2 ranks on cuda:0 (gloo-device): DDP ResNet-tiny with hook-driven overlap vs the
    single-process reference that sums both ranks' gradients."""
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.parallel.comm import GlooDeviceComm
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init(gpu_devices=[0, 0])
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    assert FluxMPI.backend_name() == "gloo-device" and FluxMPI.device().index == 0
    # MIOpen's default solvers are not run-to-run deterministic (two identical fp32 backward
    # passes of one module differed by up to 4 % of the gradient's max in a 2-block stage on
    # MI355X); the comparison below is about the communication, so pin deterministic solvers
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda", 0)
    torch.manual_seed(5 + r)  # different init per rank: DDP broadcasts rank 0's
    model = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused").to(dev, memory_format=torch.channels_last)
    torch.manual_seed(5)
    ref = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused").to(dev, memory_format=torch.channels_last)
    ddp = DDP(model, O.Descent(0.05), bucket_mb=0.5, first_bucket_mb=0.1, overlap=True)
    assert isinstance(ddp.comm, GlooDeviceComm) and ddp._hooks and len(ddp.buckets) >= 3
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.equal(p, q)  # broadcast from rank 0 at construction
    xs = [torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(10 + k)).to(dev) for k in range(W)]
    xs = [x.contiguous(memory_format=torch.channels_last) for x in xs]
    ys = [torch.randint(0, 10, (4,), generator=torch.Generator().manual_seed(20 + k)).to(dev) for k in range(W)]
    for _ in range(2):
        F.cross_entropy(ddp(xs[r]), ys[r]).backward()
        ddp.step()
        ref.zero_grad()
        for k in range(W):
            F.cross_entropy(ref(xs[k]), ys[k]).backward()
        with torch.no_grad():
            for p in ref.parameters():
                p -= 0.05 * p.grad
    torch.cuda.synchronize()
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        tol = 1e-3 * float(q.detach().abs().max()) + 1e-5
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-3, atol=tol, msg=lambda m: f"{n}: {m}")
    # the device-tensor functional paths too: bucketed allreduce + synchronize
    t = torch.full((1000,), float(r + 1), device=dev)
    FluxMPI.allreduce_gradients({"t": t})
    torch.cuda.synchronize()
    assert torch.all(t == 3.0)
    FluxMPI.synchronize(model)
    FluxMPI.Finalize()


def test_two_ranks_one_gpu_gloo_device(gpu_ext):
    from tests.conftest import run_spmd

    run_spmd("tests.test_comm_gpu:worker_two_ranks_one_gpu", nprocs=2,
             env={"FLUXMPI_BACKEND": "gloo-device"}, timeout=240)


def worker_calibrate_two_ranks():
    """Rank-consistent kernel choices at N>1 (parallel/autotune.py): rank 0 measures during a
    no_sync forward+backward with no gradient collective in flight, every rank ends with the
    identical frozen table, and later steps add nothing rank-local to it."""
    import torch.distributed as dist

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.models.resnet import ResNet
    from fluxmpi_amd.ops import fused_block
    from fluxmpi_amd.parallel.autotune import calibrate
    from fluxmpi_amd.parallel.ddp import DDP
    from fluxmpi_amd.parallel.runtime import cpu_comm

    FluxMPI.Init(gpu_devices=[0, 0])
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    model = ResNet((1, 1, 1, 1), 10, conv_impl="hybrid", norm="fused").to(dev, memory_format=torch.channels_last)
    for m in model.modules():
        if not isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and type(m).__name__ != "FusedBatchNorm2d":
            for p in m.parameters(recurse=False):
                p.data = p.data.to(torch.bfloat16)
    ddp = DDP(model, O.Adam(1e-3), bucket_mb=0.5, first_bucket_mb=0.1, overlap=True)
    x = torch.randn(8, 3, 64, 64, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    assert not fused_block.dump_choices()  # nothing measured yet
    recs = calibrate(ddp, lambda: F.cross_entropy(ddp(x).float(), y).backward())
    assert ddp.collectives_launched == 0  # the table was fixed before any gradient collective
    assert recs and fused_block.choices_frozen()
    mine = sorted(fused_block.dump_choices())
    everyone = [None, None]
    dist.all_gather_object(everyone, mine, group=cpu_comm().group)
    assert everyone[0] == everyone[1] == sorted(recs)
    for _ in range(2):
        F.cross_entropy(ddp(x).float(), y).backward()
        ddp.step()
    assert ddp.collectives_launched > 0 and sorted(fused_block.dump_choices()) == mine
    FluxMPI.Finalize()


def test_calibrate_two_ranks_one_gpu(gpu_ext):
    from tests.conftest import run_spmd

    run_spmd("tests.test_comm_gpu:worker_calibrate_two_ranks", nprocs=2,
             env={"FLUXMPI_BACKEND": "gloo-device"}, timeout=240)
