"""Launchers: our `python -m fluxmpi_amd.launch` and `torch.distributed.run` (what the driver uses)."""
import os
import subprocess
import sys

from tests.conftest import ROOT

SCRIPT = r'''
import torch, fluxmpi_amd as F
F.Init()
r, w = F.local_rank(), F.total_workers()
x = F.allreduce(torch.ones(3) * r, "+")
assert torch.equal(x, torch.full((3,), float(sum(range(w))))), x
assert F.synchronize(float(r)) == 0.0
F.fluxmpi_println("ok")
F.Finalize()
'''


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e["FLUXMPI_BACKEND"] = "gloo"
    e["GLOO_SOCKET_IFNAME"] = "lo"
    return e


def test_torchrun(tmp_path):
    from fluxmpi_amd.launch import free_port
    p = tmp_path / "prog.py"
    p.write_text(SCRIPT)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(p)],
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok") == 2


def test_fluxmpi_launch_script(tmp_path):
    p = tmp_path / "prog.py"
    p.write_text(SCRIPT)
    r = subprocess.run([sys.executable, "-m", "fluxmpi_amd.launch", "-n", "3", str(p)], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("[") >= 3


def test_launch_propagates_failure(tmp_path):
    p = tmp_path / "bad.py"
    p.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    r = subprocess.run([sys.executable, "-m", "fluxmpi_amd.launch", "-n", "2", str(p)], env=_env(), timeout=120)
    assert r.returncode == 3


def test_bench_collectives_cpu():
    """scripts/bench_collectives.py (the nccl-tests analogue) on 2 CPU ranks: one JSON line per
    (collective, size) with bus bandwidth = algorithm bandwidth x the ring factor."""
    import json
    r = subprocess.run([sys.executable, "-m", "fluxmpi_amd.launch", "-n", "2",
                        os.path.join(ROOT, "scripts", "bench_collectives.py"), "--device", "cpu", "--sizes", "4K,64K",
                        "--iters", "2", "--warmup", "1"], env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert {ln["op"] for ln in lines} == {"allreduce", "allgather", "reduce_scatter", "broadcast", "alltoall"}
    assert len(lines) == 10 and all(ln["world"] == 2 and ln["us"] > 0 for ln in lines)
    ar = [ln for ln in lines if ln["op"] == "allreduce"][0]
    assert abs(ar["busbw_GBps"] - ar["algbw_GBps"]) < 1e-2  # 2(N-1)/N == 1 at N=2
