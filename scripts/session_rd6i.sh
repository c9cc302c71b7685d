#!/bin/bash
# round 6: the 4-rank same-device rehearsal with the measured bucket plan, optimiser placement under
# emulated RCCL traffic, linbwd per-shape timings, DEQ solver iterations under training with a
# learnable synthetic task (teacher labels) and with several batches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
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
for m in deq deq_cifar; do
  for lb in random teacher; do
    for nb in 1 8; do
      step dl_${m}_${lb}_$nb 200 0 python scripts/diag_deq_contract.py --model $m --steps 40 --labels $lb --batches $nb
    done
  done
done
echo done
