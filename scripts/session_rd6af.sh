#!/bin/bash
# round 6 final check after the MNIST restart preset: whole GPU suite, smoke(), bench lines,
# DEQ --force-comm and 2-rank --same-device rehearsals
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 1000 0 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 0 python -c "import __graft_entry__ as g; g.smoke()"
B="python bench.py --steps 20 --warmup 10"
step resnet 300 0 python bench.py
step vit 300 0 $B --model vit_b16
step deq 300 0 $B --model deq
step deq_comm 300 0 $B --model deq --force-comm
step deq_cifar 300 0 $B --model deq_cifar
step deq_cifar_comm 300 0 $B --model deq_cifar --force-comm
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step deq_2rank 400 0 $R --master-port 29571 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5
step deqc_2rank 400 0 $R --master-port 29572 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5
echo done
