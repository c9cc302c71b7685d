#!/bin/bash
# round 5: GroupNorm loads in flight per lane (kU 4 / 8 / 16) at the DEQ shapes
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step gn_ku4 120 0 python scripts/bench_gn.py
step gn_ku8 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn_ku8.so python scripts/bench_gn.py
step gn_ku16 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn_ku16.so python scripts/bench_gn.py
step gn_ku4_b 120 0 python scripts/bench_gn.py
step gn_ku16_b 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn_ku16.so python scripts/bench_gn.py
echo done
