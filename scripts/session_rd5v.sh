#!/bin/bash
# round 5: N > 1 rehearsal on one GPU (ranks share the device; not a scaling number): ResNet-50,
# ViT-B/16 and DEQ-CIFAR through torchrun with 4 ranks, small per-rank batches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
step r4_resnet 400 0 $R --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 3 --batch 32 --same-device
step r4_vit 400 0 $R --master-port 29542 bench.py --gpus 4 --steps 5 --warmup 3 --batch 16 --same-device --model vit_b16
step r4_deqc 400 0 $R --master-port 29543 bench.py --gpus 4 --steps 5 --warmup 3 --batch 32 --same-device --model deq_cifar
echo done
