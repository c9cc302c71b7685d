"""Process launcher: ``python -m fluxmpi_amd.launch -n N script.py [args...]``.

The ``mpiexecjl -n N julia script.jl`` analogue (reference ``README.md:72``,
``docs/src/guide.md:21``). Spawns N ranks on this node with ``RANK``,
``WORLD_SIZE``, ``LOCAL_RANK``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR`` (127.0.0.1)
and ``MASTER_PORT`` set, streams their output, and returns the first non-zero
exit code. If one rank fails the others are terminated (by PID — only the
processes this launcher started).

``--fn module:function`` runs a Python function in every rank instead of a
script (used by the SPMD test-suite).
``torchrun``/``torch.distributed.run`` and ``mpiexec`` work as launchers too.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(nprocs: int, argv: list[str], env: dict | None = None, timeout: float | None = None,
           master_port: int | None = None) -> int:
    port = master_port or free_port()
    procs = []
    base = dict(os.environ)
    # like torchrun: avoid nprocs x all-cores OpenMP oversubscription on CPU ranks
    base.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // max(1, nprocs))))
    # the ranks import this package even when the script lives elsewhere (mpiexecjl --project)
    pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = base.get("PYTHONPATH", "").split(os.pathsep) if base.get("PYTHONPATH") else []
    if pkg_root not in paths:
        base["PYTHONPATH"] = os.pathsep.join([pkg_root] + paths)
    if env:
        base.update(env)
    for r in range(nprocs):
        e = dict(base)
        e.update({
            "RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nprocs),
            "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "GLOO_SOCKET_IFNAME": e.get("GLOO_SOCKET_IFNAME", "lo"),
        })
        procs.append(subprocess.Popen(argv, env=e))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = False
            for p in procs:
                code = p.poll()
                if code is None:
                    alive = True
                elif code != 0 and rc == 0:
                    rc = code
            if rc != 0 or not alive:
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc == 0:
        rc = max((p.returncode or 0) for p in procs)
    return rc


def _run_fn(target: str, args: list[str]) -> None:
    import importlib

    mod, fn = target.split(":")
    f = getattr(importlib.import_module(mod), fn)
    f(*args)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--nprocs", type=int, default=int(os.environ.get("FLUXMPI_TEST_NPROCS", "2")))
    ap.add_argument("--fn", help="module:function to run in every rank")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.fn:
        child = [sys.executable, "-m", "fluxmpi_amd.launch", "--_child", a.fn, *a.cmd]
    else:
        if not a.cmd:
            ap.error("nothing to run")
        cmd = a.cmd[1:] if a.cmd[0] == "--" else a.cmd
        child = [sys.executable, *cmd] if cmd[0].endswith(".py") else cmd
    return launch(a.nprocs, child, timeout=a.timeout, master_port=a.master_port)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--_child":
        _run_fn(sys.argv[2], sys.argv[3:])
        sys.exit(0)
    sys.exit(main())
