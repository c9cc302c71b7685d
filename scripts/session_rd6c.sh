#!/bin/bash
# round 6: DEQ forward-solve residual curves on the trained cells (solver / precision diagnosis)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step diag_solver_deq 300 0 python scripts/diag_deq_solver.py --model deq --train 40
step diag_solver_deqc 400 0 python scripts/diag_deq_solver.py --model deq_cifar --train 40
echo done
