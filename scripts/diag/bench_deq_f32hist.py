"""bench.py with the Anderson F history forced to fp32 (the pre-round-5 layout): the A arm of
the bf16-F-history A/B. usage: python scripts/diag/bench_deq_f32hist.py <bench.py args...>"""
import os
import runpy
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fluxmpi_amd.models import deq as D  # noqa: E402

D._f_hist_dtype = lambda dt, like: torch.float32
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
