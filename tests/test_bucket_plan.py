"""The measured gradient-bucket plan (``parallel/bucket_plan.py``): the fit and the choice on
synthetic latency / bandwidth curves, and the probe + plan inside DDP on a live gloo group (every
rank builds the same buckets; the record carries the samples)."""
import pytest
import torch

MIB = 1 << 20


def _curve(alpha_us, busbw_gbs, world=8, noise=0.0):
    from fluxmpi_amd.parallel.bucket_plan import LADDER
    g = torch.Generator().manual_seed(0)
    f = 2.0 * (world - 1) / world
    out = []
    for n in LADDER:
        t = alpha_us + f * n / (busbw_gbs * 1e3)
        out.append((n, t * (1.0 + noise * float(torch.randn((), generator=g)))))
    return out


def test_fit_recovers_latency_and_bandwidth():
    from fluxmpi_amd.parallel.bucket_plan import fit
    m = fit(_curve(25.0, 300.0), 8)
    assert m.alpha_us == pytest.approx(25.0, rel=1e-6)
    assert m.busbw_gbs() == pytest.approx(300.0, rel=1e-6)
    # a few per cent of noise moves the fit by about as much
    m = fit(_curve(25.0, 300.0, noise=0.03), 8)
    assert 15.0 < m.alpha_us < 35.0 and 270.0 < m.busbw_gbs() < 330.0


@pytest.mark.parametrize("alpha,bw,bucket,first,tail", [
    # RCCL-like over 8 xGMI-connected GPUs: n_half = 25 us * 300 GB/s / 1.75 = 4.1 MiB
    (25.0, 300.0, 16.5, 8.25, 4.0),
    # latency-bound (e.g. host-staged / gloo): n_half 5.45 MiB
    (2000.0, 5.0, 22.0, 11.0, 5.5),
    # more so: clamped at 64 MiB
    (20000.0, 5.0, 64.0, 64.0, 54.5),
    # almost free collectives: the smallest pieces
    (0.5, 1000.0, 1.25, 0.5, 0.25),
])
def test_choose_from_the_half_performance_size(alpha, bw, bucket, first, tail):
    from fluxmpi_amd.parallel.bucket_plan import choose, fit
    plan = choose(fit(_curve(alpha, bw), 8))
    assert plan["bucket_mb"] == pytest.approx(bucket, abs=0.26)
    assert plan["first_bucket_mb"] == pytest.approx(first, abs=0.26)
    assert plan["tail_bucket_mb"] == pytest.approx(tail, abs=0.26)
    assert plan["tail_bucket_mb"] <= plan["first_bucket_mb"] <= plan["bucket_mb"]
    # each full bucket runs at >= ~80 % of the asymptotic bus bandwidth unless clamped
    m = fit(_curve(alpha, bw), 8)
    if plan["bucket_mb"] < 64:
        assert m.busbw_gbs(plan["bucket_mb"] * MIB) >= 0.79 * m.busbw_gbs()


def test_choose_caps_the_bucket_count():
    from fluxmpi_amd.parallel.bucket_plan import choose, fit
    plan = choose(fit(_curve(0.5, 1000.0), 8), total_bytes=4096 * MIB)
    assert plan["bucket_mb"] >= 4096 / 64


def test_fit_degenerate_curves():
    from fluxmpi_amd.parallel.bucket_plan import fit
    flat = [(n, 100.0) for n, _ in _curve(1.0, 1.0)]  # no size dependence at all
    m = fit(flat, 4)
    assert m.beta_us_per_byte > 0 and m.alpha_us >= 0
    with pytest.raises(ValueError):
        fit([(1 << 20, 10.0)], 2)


def worker_measured_plan():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.autotune import broadcast_lines
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    torch.manual_seed(0)
    model = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(6)])
    d = DDP(model, O.Descent(0.1))
    s = d.comm_summary()
    assert s["bucket_plan"] == "measured", s
    probe = s["comm_probe"]
    assert [r["kib"] for r in probe["samples"]] == [256, 1024, 4096, 16384, 65536]
    assert all(r["us"] > 0 for r in probe["samples"])
    # every rank holds the same plan and built the same buckets
    mine = repr((probe["plan"], [b.numel for b in d.buckets]))
    assert broadcast_lines([mine])[0] == mine
    # explicit sizes win over the measurement
    d2 = DDP(model, O.Descent(0.1), bucket_mb=0.1, first_bucket_mb=0.05)
    assert d2.comm_summary()["bucket_plan"] == "default"
    x = torch.randn(4, 256)
    d(x).sum().backward()
    d.step()
    FluxMPI.Finalize()


def test_measured_plan_gloo(spmd):
    spmd("tests.test_bucket_plan:worker_measured_plan", timeout=180)


def test_probe_keeps_the_fastest_pass():
    """probe(): every ladder size keeps its fastest pass — a slow first pass (a rank arriving late at
    the first timed size, connection setup) does not reach the fit."""
    import time

    from fluxmpi_amd.parallel.bucket_plan import probe

    class SlowFirstPass:
        size = 1

        def __init__(self):
            self.calls = 0

        def allreduce(self, t):
            self.calls += 1
            # 2 warm-up + 3 timed calls per size and pass; the first pass's timed calls are slow
            if self.calls <= 2 * 5 and (self.calls - 1) % 5 >= 2:
                time.sleep(0.02)

        def barrier(self):
            pass

    sizes = (1 << 10, 1 << 12)
    out = probe(SlowFirstPass(), torch.device("cpu"), torch.float32, sizes=sizes, iters=3, warmup=2, passes=2)
    assert [n for n, _ in out] == list(sizes)
    assert all(us < 10_000 for _, us in out), out  # the 20 ms first-pass calls were dropped
