#!/bin/bash
# round 5: final validation after the 16-channel conv3x3n tail blocks (GPU suite, smoke, bench lines, ResNet-50 steady trace)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_gpu 900 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step resnet 300 0 $B
step vit 300 0 $B --model vit_b16
step deq 300 0 $B --model deq
step deq_cifar 300 0 $B --model deq_cifar --force-comm
step resnet_comm 300 0 $B --force-comm
step resnet_b 300 0 $B
cd /tmp
step prof_resnet 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_resnet_rd5ba" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd "$ROOT"
echo done
