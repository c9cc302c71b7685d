#!/bin/bash
# round 6: DEQ-CIFAR preset with Skip DEQ (skip convolution on the implicit-GEMM 3x3 kernels) —
# plain, --force-comm, 2-rank rehearsal; MNIST forward solver variants (Anderson memory 8, fp32 histories)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_deq 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py
B="python bench.py --steps 40 --warmup 10"
step c 300 0 $B --model deq_cifar
step c_comm 300 0 $B --model deq_cifar --force-comm
step m5 300 0 $B --model deq
step m8 300 0 $B --model deq --deq-solver m=8
step mh32 300 0 env FLUXMPI_DEQ_HIST=fp32 $B --model deq
step m5b 300 0 $B --model deq
step m8b 300 0 $B --model deq --deq-solver m=8
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c_2rank 400 0 $R --master-port 29561 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5
step m8_2rank 400 0 $R --master-port 29562 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5 --deq-solver m=8
echo done
