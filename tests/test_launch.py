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
