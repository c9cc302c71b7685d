"""Precision of gradient sums on the wire.

bf16 gradient buckets are summed by the collective in their own dtype (``comm_dtype="native"``,
the default): RCCL's ring reduce-scatter adds one rank's chunk per hop and stores the partial sum
back in bf16, so an 8-rank sum carries up to 7 roundings on top of the one each gradient already
had when the backward wrote it. The reference sums Float32 and checks to 1e-5
(``/root/reference/test/test_optimizer.jl:20-26``).

What these tests pin down:

* an emulated ring (sequential bf16 accumulation, the order a ring hop applies) at 2 / 4 / 8
  ranks: the relative L2 error of the bf16-wire sum against the exact sum of the same bf16
  gradients stays within ``1.25 sqrt(W - 1)`` times ONE bf16 rounding of the exact sum (the hops'
  roundings add up like independent errors); measured 0.19 / 0.25 / 0.32 % at 2 / 4 / 8 ranks
  against 0.17 % for one rounding, so under 2^-8 at 8 ranks — the size of the bf16 rounding the
  gradient itself already carries relative to its fp32 value;
* the fp32 wire (``FLUXMPI_COMM_DTYPE=fp32``) meets the reference's 1e-5;
* the same bound on a live 8-rank gloo group through the engine's bucket path, where the fp32
  wire leaves exactly one bf16 rounding (the reduced sum lands back in the bf16 gradient bucket).

Decision recorded from them: ``native`` stays the default for bf16 models (half the bytes per
collective; the optimiser's fp32 master weights and Adam's normalised step absorb a ~0.5 %
gradient perturbation, the same order as the bf16 gradient itself); ``fp32`` is the setting
for runs that must match an fp32 reference sum to 1e-5, as the reference's tests do.
"""
import math

import pytest
import torch


def _grads(world, n=1 << 16, seed=0):
    g = torch.Generator().manual_seed(seed)
    common = torch.randn(n, generator=g)  # ranks' gradients are correlated (same model, similar data)
    return [(0.7 * common + 0.7 * torch.randn(n, generator=g)).bfloat16() for _ in range(world)]


def _ring_sum(parts, dtype):
    acc = parts[0].to(dtype)
    for p in parts[1:]:
        acc = (acc.float() + p.float()).to(dtype)  # one hop: add in fp32, store in the wire dtype
    return acc


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ring_sum_error_bf16_vs_fp32_wire(world):
    parts = _grads(world)
    exact = torch.stack([p.double() for p in parts]).sum(0)
    e16 = _rel(_ring_sum(parts, torch.bfloat16), exact)
    e32 = _rel(_ring_sum(parts, torch.float32), exact)
    one = _rel(exact.bfloat16(), exact)  # one bf16 rounding of the exact sum, for scale
    assert e16 < 1.25 * math.sqrt(world - 1) * one, (world, e16, one)
    assert e16 >= 0.9 * one  # the rounding is real (the test measures something)
    if world == 8:
        assert e16 < 2.0 ** -8
    assert e32 < 1e-6  # the fp32 wire meets the reference's 1e-5 with room


def worker_wire_8():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    r, W = FluxMPI.local_rank(), FluxMPI.total_workers()
    parts = _grads(W, n=1 << 14)
    exact = torch.stack([p.double() for p in parts]).sum(0)
    for dt, tol in ((torch.bfloat16, 2.0 ** -8), (torch.float32, 1e-5)):
        t = parts[r].to(dt, copy=True)
        FluxMPI.allreduce(t, "+")
        assert _rel(t, exact) < tol, (dt, _rel(t, exact))
    # through the engine: a bf16 parameter whose gradient is this rank's part; Descent(1) applies
    # the reduced sum, so the update is the wire sum
    one = _rel(exact.bfloat16(), exact)
    # bf16 wire: the ring's roundings; fp32 wire: the sum is exact in fp32 and rounded ONCE, when
    # it lands back in the bf16 gradient bucket the optimiser reads
    for cd, tol in ((None, 2.0 ** -8), (torch.float32, 1.01 * one)):
        p = torch.nn.Parameter(torch.zeros(1 << 14, dtype=torch.bfloat16))
        m = torch.nn.Module()
        m.p = p
        d = DDP(m, O.Descent(1.0), comm_dtype=cd, master_weights=True, bucket_mb=1, first_bucket_mb=1)
        (p.float() * parts[r].float()).sum().backward()
        d.step()
        upd = -d.buckets[0].master[: p.numel()]  # fp32 master: no final bf16 rounding of the update
        e = _rel(upd, exact)
        assert e < tol, (cd, e)
    FluxMPI.Finalize()


def test_wire_precision_8_ranks_gloo(spmd):
    spmd("tests.test_wire_precision:worker_wire_8", nprocs=8, timeout=240)
