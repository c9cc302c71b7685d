#!/bin/bash
# round 5: --force-comm steady traces on the final tree (ResNet-50, DEQ-CIFAR, ViT-B/16): do any pack
# copies (mt_copy) or runtime buffer copies remain in the steady step?
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
cd /tmp
for m in resnet50 deq_cifar vit_b16; do
  step prof_fc_$m 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fc_${m}_rd5aw" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --model $m --steps 5 --warmup 5 --force-comm
done
cd "$ROOT"
echo done
