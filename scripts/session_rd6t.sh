#!/bin/bash
# round 6: Skip DEQ under communication (--force-comm, 2-rank --same-device rehearsals) and a longer
# MNIST window (the rd6s MNIST bench lines disagreed with the 40-step diag runs)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
S="--deq-solver skip=1,skip_reg=1"
B="python bench.py --steps 20 --warmup 10"
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step deqc_sk1_comm 300 0 $B --model deq_cifar --force-comm $S
step deqc_sk1_2rank 400 0 $R --master-port 29541 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5 $S
step deqc_sk0_2rank 400 0 $R --master-port 29542 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5
step deq_sk1_2rank 400 0 $R --master-port 29543 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5 $S
step deq_sk1_long 300 0 python bench.py --steps 40 --warmup 10 --model deq $S
step deq_sk0_long 300 0 python bench.py --steps 40 --warmup 10 --model deq
echo done
