#!/bin/bash
# round 6: DEQ forward-solve residual curves on the trained cells (solver / precision diagnosis);
# conv_c3 filter gradient with the pipelined dY loads (test + DEQ-CIFAR profile); roofline BatchNorm
# rows timed by graph replay
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step test_c3 300 0 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_c3_gpu.py
step roofline_bn 300 0 env ROOFLINE_BN_ONLY=1 python scripts/roofline_resnet50.py "$OUT/rd6c_roofline_bn.md"
cd /tmp
step prof_deqc 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deqc_rd6c" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5 --force-comm
cd "$ROOT"
step diag_solver_deq 300 0 python scripts/diag_deq_solver.py --model deq --train 40
step diag_solver_deqc 400 0 python scripts/diag_deq_solver.py --model deq_cifar --train 40
echo done
