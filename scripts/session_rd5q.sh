#!/bin/bash
# round 5: wgrad3x3n diagnostics — staging alone, compute alone
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step t_base 120 0 python scripts/diag/time_w3n.py
step t_noload 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_w3n_noload.so python scripts/diag/time_w3n.py
step t_nocompute 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_w3n_nocompute.so python scripts/diag/time_w3n.py
step t_base2 120 0 python scripts/diag/time_w3n.py
echo done
