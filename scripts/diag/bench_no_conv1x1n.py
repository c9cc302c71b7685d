"""bench.py with the narrow-K 1x1 forward kernel switched off (the previous routing): the A arm of
the conv1x1n A/B. usage: python scripts/diag/bench_no_conv1x1n.py <bench.py args...>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fluxmpi_amd.ops import gemm as G  # noqa: E402

G.conv1x1n_ok = lambda *a, **k: False
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
