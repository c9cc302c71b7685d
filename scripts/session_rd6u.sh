#!/bin/bash
# round 6: the adjoint solve by Anderson (bwd_m = 5, per-sample normalised right-hand side) vs the
# fixed-point adjoint, on the DEQ and DEQ-CIFAR (Skip DEQ) bench lines and 2-rank rehearsals
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_deq 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py
B="python bench.py --steps 40 --warmup 10"
step m_p 300 0 $B --model deq
step m_a5 300 0 $B --model deq --deq-solver bwd_m=5,bwd_tol=5e-3
step m_a10 300 0 $B --model deq --deq-solver bwd_m=5,bwd_tol=1e-2
step c_p 300 0 $B --model deq_cifar --deq-solver skip=1
step c_a3 300 0 $B --model deq_cifar --deq-solver skip=1,bwd_m=5,bwd_tol=3e-3
step m_p2 300 0 $B --model deq
step m_a52 300 0 $B --model deq --deq-solver bwd_m=5,bwd_tol=5e-3
step c_p2 300 0 $B --model deq_cifar --deq-solver skip=1
step c_a32 300 0 $B --model deq_cifar --deq-solver skip=1,bwd_m=5,bwd_tol=3e-3
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step m_a5_2rank 400 0 $R --master-port 29551 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5 --deq-solver bwd_m=5,bwd_tol=5e-3
step c_a3_2rank 400 0 $R --master-port 29552 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5 --deq-solver skip=1,bwd_m=5,bwd_tol=3e-3
echo done
