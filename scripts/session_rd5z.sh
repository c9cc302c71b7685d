#!/bin/bash
# round 5: steady-state kernel traces of the current tree (ResNet-50, DEQ-CIFAR with bf16 Anderson
# histories, DEQ)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
cd /tmp
step prof_resnet 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_resnet_rd5z" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 5
step prof_deq_cifar 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_cifar_rd5z" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5 --force-comm
step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_rd5z" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5
cd "$ROOT"
echo done
