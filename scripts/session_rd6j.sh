#!/bin/bash
# round 6: DEQ bench lines whose solves end by tolerance (caps raised to 60, relative tolerances
# 1e-2 MNIST / 2e-2 CIFAR, adjoint 1e-2), with and without Jacobian regularisation, against the
# capped defaults; ViT-B/16 steady trace of the round-6 routing (linbwd backward)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --steps 20 --warmup 10"
SM="max_iter=60,tol=1e-2,bwd_iter=60,bwd_tol=1e-2"
SC="max_iter=60,tol=2e-2,bwd_iter=60,bwd_tol=1e-2"
step deq_conv 300 0 $B --model deq --deq-solver $SM
step deqc_conv 300 0 $B --model deq_cifar --deq-solver $SC
step deq_conv_jr 300 0 env FLUXMPI_DEQ_JR=2.0,0.05 $B --model deq --deq-solver $SM
step deqc_conv_jr 300 0 env FLUXMPI_DEQ_JR=2.0,0.05 $B --model deq_cifar --deq-solver $SC
step deq_def 300 0 $B --model deq
step deqc_def 300 0 $B --model deq_cifar
cd /tmp
step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd6j" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
