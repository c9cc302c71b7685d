#!/bin/bash
# round 5: N > 1 rehearsal on the final tree (2 ranks on one GPU over the gloo device communicator)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step r2_resnet 400 0 $R --master-port 29551 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --same-device
step r2_vit 400 0 $R --master-port 29552 bench.py --gpus 2 --steps 5 --warmup 3 --batch 32 --same-device --model vit_b16
step r2_deqc 400 0 $R --master-port 29553 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --same-device --model deq_cifar
echo done
