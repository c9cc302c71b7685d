#!/bin/bash
# round 6 final rehearsals of the N > 1 path on one GPU (--same-device): ResNet-50 at 4 ranks, ViT-B/16
# at 2 ranks, measured bucket plan and the communicator self-report in the bench line
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step resnet_4rank 600 0 $R --nproc-per-node 4 --master-port 29581 bench.py --gpus 4 --same-device --steps 5 --warmup 3
step vit_2rank 600 0 $R --nproc-per-node 2 --master-port 29582 bench.py --gpus 2 --same-device --model vit_b16 --steps 5 --warmup 3
echo done
