#!/bin/bash
# round 5: forward residual vs iterations with fp32 / bf16 Anderson X and G histories (random-init models)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step r_dc_fp32 300 0 python scripts/diag/deq_residual.py --model deq_cifar
step r_dc_bf16 300 0 env FLUXMPI_DEQ_HIST=bf16 python scripts/diag/deq_residual.py --model deq_cifar
step r_d_fp32 300 0 python scripts/diag/deq_residual.py --model deq
step r_d_bf16 300 0 env FLUXMPI_DEQ_HIST=bf16 python scripts/diag/deq_residual.py --model deq
echo done
