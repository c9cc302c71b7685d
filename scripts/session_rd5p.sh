#!/bin/bash
# round 5: wgrad3x3n diagnostics — the price of the halo rows and of the fp32 partials
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step t_base 120 0 python scripts/diag/time_w3n.py
step t_nohalo 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_w3n_nohalo.so python scripts/diag/time_w3n.py
step t_nostore 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_w3n_nostore.so python scripts/diag/time_w3n.py
step t_base2 120 0 python scripts/diag/time_w3n.py
echo done
