#!/bin/bash
# round 6: DEQ Jacobian regularisation (per-step solver iterations / residuals under training, and the
# trained cells' residual curves), linbwd with the measured split choice (tests, ViT A/B), the 4-rank
# same-device rehearsal with the measured bucket plan, optimiser placement under emulated RCCL traffic
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_lb 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linbwd_gpu.py
for jr in 0.5,0.05 2.0,0.05; do
  step jr_deq_$jr 200 0 env FLUXMPI_DEQ_JR=$jr python scripts/diag_deq_contract.py --model deq --steps 40
  step jr_deqc_$jr 300 0 env FLUXMPI_DEQ_JR=$jr python scripts/diag_deq_contract.py --model deq_cifar --steps 40
done
step jrsolver_deq 300 0 env FLUXMPI_DEQ_JR=2.0,0.05 python scripts/diag_deq_solver.py --model deq --train 40
B="python bench.py --steps 20 --warmup 10"
step vit_lb1 300 0 $B --model vit_b16
step vit_lb0 300 0 env FLUXMPI_LINBWD=0 $B --model vit_b16
step vit_lb1b 300 0 $B --model vit_b16
step vit_lb0b 300 0 env FLUXMPI_LINBWD=0 $B --model vit_b16
step bench_linbwd 300 0 python scripts/bench_linbwd.py
step rehearsal4 600 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 4 --same-device --steps 5 --warmup 3
BF="python bench.py --steps 20 --warmup 10 --force-comm"
for m in vit_b16 resnet50; do
  step emu_ov1_$m 300 0 $BF --model $m --emulate-comm 64:300 --overlap-opt 1
  step emu_ov0_$m 300 0 $BF --model $m --emulate-comm 64:300 --overlap-opt 0
  step emu_ov1b_$m 300 0 $BF --model $m --emulate-comm 64:300 --overlap-opt 1
  step emu_ov0b_$m 300 0 $BF --model $m --emulate-comm 64:300 --overlap-opt 0
done
echo done
