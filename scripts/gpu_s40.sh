#!/bin/bash
# session 40: A/B of the BN-backward epilogue link (FLUXMPI_BN_LINK=1) on the current pipeline
source "$(dirname "$0")/gpu_lib.sh"
step bench_bnlink 400 0 env FLUXMPI_BN_LINK=1 python bench.py
step bench_default 400 0 python bench.py
step bench_bnlink2 400 0 env FLUXMPI_BN_LINK=1 python bench.py
echo done
