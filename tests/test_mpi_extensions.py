"""Mirror of reference test/test_mpi_extensions.jl (comm primitives), plus extras."""
import numpy as np


def _rank_array(shape, root_rank=0):
    import torch
    import fluxmpi_amd as FluxMPI
    return torch.ones(shape, dtype=torch.float64) if FluxMPI.local_rank() == root_rank else torch.zeros(
        shape, dtype=torch.float64)


def worker():
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import COMM_WORLD

    FluxMPI.Init(verbose=True)
    W = FluxMPI.total_workers()
    r = FluxMPI.local_rank()

    # --- Iallreduce! (out of place)
    x = torch.ones(4, dtype=torch.float64)
    y = torch.empty_like(x)
    y, req = FluxMPI.Iallreduce(x, y, "+", COMM_WORLD)
    FluxMPI.Wait(req)
    assert torch.equal(y, x * W)
    y = torch.empty_like(x)
    y, req = FluxMPI.Iallreduce(x, y, "*")
    req.wait()
    assert torch.equal(y, x)
    # in place form
    z = torch.full((3,), float(r + 1))
    z, req = FluxMPI.Iallreduce(z, max)
    FluxMPI.Waitall([req])
    assert torch.equal(z, torch.full((3,), float(W)))

    # --- Ibcast!
    x = _rank_array((2, 3), 0)
    y, req = FluxMPI.Ibcast(x, 0, COMM_WORLD)
    FluxMPI.Wait(req)
    assert torch.equal(y, torch.ones(2, 3, dtype=torch.float64))

    # --- blocking wrappers
    x = torch.ones(4)
    assert torch.equal(FluxMPI.allreduce(x.clone(), "+", COMM_WORLD), x * W)
    assert torch.equal(FluxMPI.allreduce(x.clone(), "*", COMM_WORLD), x)
    x = _rank_array((2, 3), 0)
    assert torch.equal(FluxMPI.bcast(x.clone(), 0, COMM_WORLD), torch.ones(2, 3, dtype=torch.float64))
    x = torch.ones(4)
    y = FluxMPI.reduce(x.clone(), "+", 0, COMM_WORLD)
    if r == 0:
        assert torch.equal(y, x * W)
    else:
        assert torch.equal(y, x)

    # --- extras: numpy buffers (in place), scalars, min/avg, ints, non-contiguous
    a = np.ones(5, dtype=np.float32)
    FluxMPI.allreduce(a, "+")
    assert np.all(a == W)
    assert FluxMPI.allreduce(float(r), "+") == sum(range(W))
    assert FluxMPI.allreduce([r, 1], "+") == [sum(range(W)), W]
    assert torch.equal(FluxMPI.allreduce(torch.tensor([r]), min), torch.tensor([0]))
    assert torch.allclose(FluxMPI.allreduce(torch.tensor([float(r)]), "avg"), torch.tensor([(W - 1) / 2]))
    m = torch.ones(4, 4)[:, ::2]
    FluxMPI.allreduce(m, "+")
    assert torch.equal(m, torch.full((4, 2), float(W)))
    g = FluxMPI.allgather(torch.tensor([float(r)]))
    assert torch.equal(g.reshape(-1), torch.arange(W, dtype=torch.float32))
    rs = FluxMPI.reduce_scatter(torch.ones(W * 2))
    assert torch.equal(rs, torch.full((2,), float(W)))
    FluxMPI.Finalize()


def test_mpi_extensions(spmd):
    spmd("tests.test_mpi_extensions:worker")


def worker_four():
    worker()


def test_mpi_extensions_4ranks(spmd):
    spmd("tests.test_mpi_extensions:worker_four", nprocs=4)


def test_op_coercion():
    import operator
    from fluxmpi_amd.parallel.comm import ReduceOp, to_op
    assert to_op(operator.add) == ReduceOp.SUM
    assert to_op("+") == ReduceOp.SUM
    assert to_op(operator.mul) == ReduceOp.PROD
    assert to_op(max) == ReduceOp.MAX and to_op(min) == ReduceOp.MIN
    import pytest
    with pytest.raises(ValueError):
        to_op("xor")


def worker_rccl_bootstrap():
    """The N>1 RCCL bootstrap logic on CPU (no GPU, no RCCL): rank 0's unique id reaches every
    rank through the host store, and each Init generation (Init -> Finalize -> Init on a
    surviving store) gets a fresh id — a late rank can never pick up the previous one."""
    import os
    import time

    import torch.distributed as dist

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel.comm import bootstrap_unique_id

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    store = dist.distributed_c10d._get_default_store()
    made = []

    def make_uid():  # the ncclGetUniqueId stand-in: only rank 0 may call it
        assert r == 0
        made.append(os.urandom(128))
        return made[-1]

    seen = []
    for gen in range(3):
        if r == W - 1:
            time.sleep(0.2 * gen)  # a straggler: the others already wait on the next generation
        uid = bootstrap_unique_id(make_uid, store, r, W, tag="test")
        assert isinstance(uid, bytes) and len(uid) == 128
        seen.append(uid)
        store.set(f"check/{gen}/{r}", uid)
        FluxMPI.barrier()  # ncclCommInitRank is collective: generation k ends on every rank first
    assert len(set(seen)) == 3  # a new id per generation
    for gen in range(3):
        ids = {bytes(store.get(f"check/{gen}/{k}")) for k in range(W)}
        assert ids == {seen[gen]}  # every rank got rank 0's id of that generation
    if r == 0:
        assert made == seen
    # another tag is an independent sequence
    other = bootstrap_unique_id(make_uid, store, r, W, tag="other")
    assert other not in seen
    FluxMPI.barrier()
    FluxMPI.Finalize()


def test_rccl_bootstrap_cpu(spmd):
    spmd("tests.test_mpi_extensions:worker_rccl_bootstrap", nprocs=3, timeout=120)


class _FakeRcclHandle:
    """Stand-in for ``fluxmpi_amd._C.RcclComm``: reports a configurable rank count."""

    def __init__(self, count, rank, device=0):
        self._c, self._r, self._d = count, rank, device

    def comm_count(self):
        return self._c

    def comm_user_rank(self):
        return self._r

    def comm_device(self):
        return self._d


def _stub_rccl(rank, size, count):
    from fluxmpi_amd.parallel.comm import RcclComm

    c = object.__new__(RcclComm)  # no HIP stream / RCCL init on the CPU: only the report path
    c.rank, c.size, c.abort_reason = rank, size, None
    c._h = _FakeRcclHandle(count, rank)
    c.priority, c.version = 0, 22706
    return c


def worker_bench_selfcheck():
    """bench.py's communicator self-check on 2 gloo ranks with a stubbed native communicator:
    a rank count that is not WORLD_SIZE on ONE rank makes every rank return exit code 4 (no
    number, no hang); the matching report passes and is what the JSON line records."""
    import importlib.util
    import os

    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.parallel import runtime

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    real = runtime.device_comm
    try:
        runtime.device_comm = lambda: _stub_rccl(r, W, W if r == 0 else W - 1)  # rank 1 disagrees
        assert bench.selfcheck_or_code(FluxMPI, W, r, None) == 4
        runtime.device_comm = lambda: _stub_rccl(r, W, W)
        rep = bench.selfcheck_or_code(FluxMPI, W, r, None)
        assert rep["rccl_nranks"] == W and rep["rccl_rank"] == r and rep["comm_priority"] == 0
        # the --same-device rehearsal backend (gloo on device tensors) answers from its group
        from fluxmpi_amd.parallel.comm import GlooDeviceComm
        gd = GlooDeviceComm(runtime.cpu_comm().group, r, W)
        runtime.device_comm = lambda: gd
        rep = bench.selfcheck_or_code(FluxMPI, W, r, None)
        assert rep["comm_backend"] == "gloo-device" and rep["comm_nranks"] == W and rep["comm_rank"] == r
        assert bench.selfcheck_or_code(FluxMPI, W + 1, r, None) == 4  # WORLD_SIZE disagrees
    finally:
        runtime.device_comm = real
    FluxMPI.Finalize()


def test_bench_comm_selfcheck_cpu(spmd):
    spmd("tests.test_mpi_extensions:worker_bench_selfcheck", timeout=120)
