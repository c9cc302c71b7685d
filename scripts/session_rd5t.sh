#!/bin/bash
# round 5: attention forward with K and V through one LDS buffer (FLUXMPI_ATTN_FWD=seq): numerics,
# parts sweep vs the resident kernel
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step pytest_attn_seq 300 1 env FLUXMPI_ATTN_FWD=seq python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step a_res 120 0 python scripts/bench_attn.py
for p in 2 3 4 5 7; do step a_seq$p 120 0 env FLUXMPI_ATTN_FWD=seq FLUXMPI_ATTN_SEQ_PARTS=$p python scripts/bench_attn.py; done
step a_res2 120 0 python scripts/bench_attn.py
echo done
