#!/bin/bash
# round 5: kernel traces with and without the RCCL CU-footprint emulation (ResNet-50, ViT-B/16, --force-comm)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
cd /tmp
for m in resnet50 vit_b16; do
step prof_${m}_comm 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${m}_comm_rd5ac" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model $m --steps 5 --warmup 5 --force-comm
step prof_${m}_emu 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${m}_emu_rd5ac" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model $m --steps 5 --warmup 5 --force-comm --emulate-comm 64:150:512:32
done
cd "$ROOT"
echo done
