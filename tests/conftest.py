"""Test configuration.

* ``@pytest.mark.gpu`` marks tests that need an MI355X (run on the GPU box
  with ``pytest -m gpu``); everything else runs on CPU.
* :func:`run_spmd` mirrors the reference's test driver (``test/runtests.jl``):
  a test body is an SPMD program executed by N ranks over the gloo backend
  (default ``FLUXMPI_TEST_NPROCS``, else ``clamp(cpu_count, 2, 4)`` exactly as the
  reference's driver, ``/root/reference/test/runtests.jl:3-4``: 4 on CI machines);
  assertions run inside every rank and the parent checks the exit codes. Tests
  that need a specific world (3-rank uneven shards, 8-rank wire sums, GPU
  rehearsals) pass ``nprocs`` explicitly.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")
    if os.environ.get("FLUXMPI_C_VARIANT"):  # run the suite against a variant build of the library
        sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
        import load_variant

        load_variant.install()


def default_nprocs() -> int:
    """``FLUXMPI_TEST_NPROCS`` or ``clamp(cpu_count, 2, 4)`` (the reference's ``runtests.jl:4``)."""
    v = os.environ.get("FLUXMPI_TEST_NPROCS")
    return int(v) if v else max(2, min(4, os.cpu_count() or 2))


def run_spmd(target: str, nprocs: int | None = None, env: dict | None = None, timeout: float = 300.0):
    from fluxmpi_amd.launch import launch

    n = nprocs or default_nprocs()
    e = {
        "PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
        "FLUXMPI_BACKEND": "gloo",
        "OMP_NUM_THREADS": "1",
    }
    if env:
        e.update(env)
    rc = launch(n, [sys.executable, "-m", "fluxmpi_amd.launch", "--_child", target], env=e, timeout=timeout)
    assert rc == 0, f"SPMD program {target} failed on {n} ranks (exit code {rc})"


@pytest.fixture
def spmd():
    return run_spmd


@pytest.fixture(scope="session")
def gpu_ext():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fluxmpi_amd.ops import _ext

    return _ext.get(required=True)
