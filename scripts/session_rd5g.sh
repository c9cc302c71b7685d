#!/bin/bash
# round 5: MFMA shape probe (16x16x32 vs 32x32x16 under load), same-box A/Bs of the optimiser
# overlap under --force-comm, the ResNet-50 per-op roofline on the current kernels
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step build_probe 120 0 hipcc --offload-arch=gfx950 -O3 scripts/probe/mfma_shape.hip -o /tmp/mfma_shape
step mfma_shape 120 0 /tmp/mfma_shape 200000
step resnet 300 0 $B
step resnet_comm_ov 300 0 $B --force-comm
step resnet_comm_noov 300 0 $B --force-comm --overlap-opt 0
step vit 300 0 $B --model vit_b16
step vit_comm_ov 300 0 $B --model vit_b16 --force-comm
step vit_comm_noov 300 0 $B --model vit_b16 --force-comm --overlap-opt 0
step resnet_b 300 0 $B
step vit_b 300 0 $B --model vit_b16
step roofline_r50 600 0 python scripts/roofline_resnet50.py gpurun_out/roofline_r50.md
echo done
