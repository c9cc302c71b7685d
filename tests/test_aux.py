"""Aux subsystems: replica/structure checks, watchdog, checkpointing, profiling."""
import time

import pytest
import torch


def worker_checks():
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd.utils.debug import (CollectiveMismatchError, ReplicaDivergenceError, check_replicas,
                                         check_same_structure)
    FluxMPI.Init()
    r = FluxMPI.local_rank()
    tree = {"w": torch.full((3, 3), float(r)), "b": torch.ones(2)}
    try:
        check_replicas(tree)
        raise AssertionError("divergence not detected")
    except ReplicaDivergenceError:
        pass
    tree = FluxMPI.synchronize(tree)
    check_replicas(tree)
    check_same_structure({"a": torch.ones(2)})
    bad = {"a": torch.ones(2)} if r == 0 else {"a": torch.ones(3)}
    try:
        check_same_structure(bad)
        raise AssertionError("structure mismatch not detected")
    except CollectiveMismatchError:
        pass
    FluxMPI.Finalize()


def test_replica_and_structure_checks(spmd):
    spmd("tests.test_aux:worker_checks")


def test_watchdog_detects_async_error():
    from fluxmpi_amd.utils.debug import Watchdog

    class FakeComm:
        def __init__(self):
            self.fail = False

        def check_async_error(self):
            if self.fail:
                raise RuntimeError("RCCL asynchronous error 3")

    c = FakeComm()
    wd = Watchdog(c, timeout_s=100, interval_s=0.01)
    wd.check()
    c.fail = True
    time.sleep(0.2)
    with pytest.raises(RuntimeError, match="watchdog"):
        wd.check()
    wd.stop()


def test_watchdog_timeout():
    from fluxmpi_amd.parallel.comm import Work
    from fluxmpi_amd.utils.debug import Watchdog

    class Never(Work):
        def is_completed(self):
            return False

    class OK:
        def check_async_error(self):
            pass

    wd = Watchdog(OK(), timeout_s=0.05, interval_s=0.01)
    wd.track(Never(), "allreduce bucket 0")
    time.sleep(0.3)
    with pytest.raises(RuntimeError, match="did not complete"):
        wd.check()


def test_checkpoint_roundtrip(tmp_path):
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.utils import checkpoint
    ps = {"a": torch.randn(3, 4), "nested": (torch.randn(2), 5, "name")}
    st = O.setup(O.Adam(1e-3), ps)
    st, ps = O.update(st, ps, {"a": torch.ones(3, 4), "nested": (torch.ones(2), None, None)})
    path = str(tmp_path / "ck.pt")
    checkpoint.save(path, {"ps": ps, "st": st, "step": 7})
    ps2 = {"a": torch.zeros(3, 4), "nested": (torch.zeros(2), 0, "x")}
    st2 = O.setup(O.Adam(1e-3), ps2)
    out = checkpoint.load(path, like={"ps": ps2, "st": st2, "step": 0})
    assert torch.equal(ps2["a"], ps["a"]) and out["step"] == 7
    assert torch.equal(st2["a"].state[0], st["a"].state[0])
    assert out["st"]["a"].state[2] == st["a"].state[2]
    raw = torch.load(path, weights_only=True)  # loadable without unpickling code
    assert "ps" in raw


def test_ddp_state_dict_roundtrip(tmp_path):
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.parallel.ddp import DDP
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.Linear(8, 1))
    ddp = DDP(m, O.Adam(1e-2))
    x = torch.randn(5, 4)
    m(x).sum().backward()
    ddp.step()
    sd = ddp.state_dict()
    torch.save(sd, tmp_path / "d.pt")
    m2 = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.Linear(8, 1))
    ddp2 = DDP(m2, O.Adam(1e-2))
    ddp2.load_state_dict(torch.load(tmp_path / "d.pt", weights_only=True))
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    m(x).sum().backward(); ddp.step()
    m2(x).sum().backward(); ddp2.step()
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_step_timer_and_ranges():
    from fluxmpi_amd.utils.profiling import StepTimer, range as prange
    t = StepTimer(torch.device("cpu"))
    with t.phase("fwd"):
        with prange("fwd", force=True):
            torch.randn(100, 100) @ torch.randn(100, 100)
    s = t.summary()
    assert "fwd" in s and s["fwd"] >= 0


def test_watchdog_pause_resume_stop():
    """pause() returns with no poll running and none starting; stop_all() (Finalize) stops it."""
    import time
    from fluxmpi_amd.utils import debug

    class FakeComm:
        polls = 0

        def check_async_error(self):
            FakeComm.polls += 1

    class FakeWork:
        def is_completed(self):
            raise AssertionError("polled while paused")

    wd = debug.Watchdog(FakeComm(), timeout_s=60, interval_s=0.01)
    time.sleep(0.05)
    assert FakeComm.polls > 0
    wd.pause()
    n = FakeComm.polls
    wd.track(FakeWork())  # tracked during "capture": ignored
    time.sleep(0.05)
    assert FakeComm.polls == n and wd.error is None
    wd.resume()
    time.sleep(0.05)
    assert FakeComm.polls > n
    debug.stop_all()
    assert not wd._thread.is_alive()
    n = FakeComm.polls
    time.sleep(0.03)
    assert FakeComm.polls == n


def test_watchdog_abort_marks_comm():
    """On a timeout the watchdog calls comm.abort(reason); later collectives must fail loudly."""
    import time
    from fluxmpi_amd.utils import debug

    class FakeComm:
        reason = None

        def check_async_error(self):
            pass

        def abort(self, reason):
            FakeComm.reason = reason

    class Stuck:
        def is_completed(self):
            return False

    wd = debug.Watchdog(FakeComm(), timeout_s=0.0, interval_s=0.01)
    wd.track(Stuck(), "allreduce of bucket 0")
    for _ in range(200):
        if wd.error is not None:
            break
        time.sleep(0.01)
    assert isinstance(wd.error, TimeoutError) and "bucket 0" in FakeComm.reason
    try:
        wd.check()
    except RuntimeError as e:
        assert "watchdog" in str(e)
    else:
        raise AssertionError
    wd.stop()


def worker_calibrate_cpu():
    """autotune.calibrate on 2 CPU ranks: the root's choice table (injected here, CPU ops measure
    nothing) reaches every rank, the tables freeze, and no gradient collective was launched."""
    import torch
    import fluxmpi_amd as FluxMPI
    from fluxmpi_amd import optimisers as O
    from fluxmpi_amd.ops import fused_block
    from fluxmpi_amd.parallel.autotune import calibrate
    from fluxmpi_amd.parallel.ddp import DDP

    FluxMPI.Init()
    r = FluxMPI.local_rank()
    m = torch.nn.Linear(4, 2)
    ddp = DDP(m, O.Descent(0.1))

    def fwd_bwd():
        fused_block._FWD1_CHOICE[(256, 64, 56, 56, 256)] = r == 0  # "measured" on the root only
        fused_block._WG_CHOICE[("3x3", (256, 64, 56, 56), 64)] = ("ours", (2, 512))
        ddp(torch.ones(3, 4)).sum().backward()

    calibrate(ddp, fwd_bwd)
    assert ddp.collectives_launched == 0 and fused_block.choices_frozen()
    assert fused_block._FWD1_CHOICE[(256, 64, 56, 56, 256)] is True
    assert fused_block._WG_CHOICE[("3x3", (256, 64, 56, 56), 64)] == ("ours", (2, 512))
    assert all(p.grad is None for p in m.parameters())  # calibration gradients discarded
    fused_block.freeze_choices(False)
    FluxMPI.Finalize()


def test_calibrate_cpu(spmd):
    spmd("tests.test_aux:worker_calibrate_cpu", timeout=120)
