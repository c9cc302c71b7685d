"""bench.py on a variant build of the native library (scripts/diag/build_variant.py):
    FLUXMPI_C_VARIANT=exp/variants/_C_x.so python scripts/diag/bench_variant.py <bench.py args...>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import load_variant  # noqa: E402

if load_variant.install() is None:
    sys.exit("bench_variant.py: set FLUXMPI_C_VARIANT")
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
