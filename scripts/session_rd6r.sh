#!/bin/bash
# round 6: DEQ presets with 80-iteration caps (bench lines, --force-comm, 2-rank rehearsals)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --steps 20 --warmup 10"
step deq 300 0 $B --model deq
step deq_cifar 300 0 $B --model deq_cifar
step deq_comm 300 0 $B --model deq --force-comm
step deq_cifar_comm 300 0 $B --model deq_cifar --force-comm
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step deq_2rank 400 0 $R --master-port 29531 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5
step deqc_2rank 400 0 $R --master-port 29532 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5
echo done
