#!/bin/bash
# round 6: baseline on this round's boxes (ResNet-50, ViT-B/16, DEQ, DEQ-CIFAR bench lines) and the
# ViT Linear weight gradients on a side stream (FLUXMPI_WGRAD_STREAM) A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step resnet 300 0 $B
step vit_ws0 300 0 env FLUXMPI_WGRAD_STREAM=0 $B --model vit_b16
step vit_ws1 300 0 env FLUXMPI_WGRAD_STREAM=1 $B --model vit_b16
step vit_ws0b 300 0 env FLUXMPI_WGRAD_STREAM=0 $B --model vit_b16
step vit_ws1b 300 0 env FLUXMPI_WGRAD_STREAM=1 $B --model vit_b16
step deq 300 0 $B --model deq
step deq_cifar 300 0 $B --model deq_cifar --force-comm
echo done
