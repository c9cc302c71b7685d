#!/bin/bash
# session 43: same-box A/B of the XCD-aware weight-gradient grid order
source "$(dirname "$0")/gpu_lib.sh"
step bench_remap1 400 0 python bench.py
step bench_remap0 400 0 env FLUXMPI_WGRAD_REMAP=0 python bench.py
step bench_remap1b 400 0 python bench.py
step bench_remap0b 400 0 env FLUXMPI_WGRAD_REMAP=0 python bench.py
echo done
