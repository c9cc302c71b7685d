#!/bin/bash
# round 6: (a) 4-rank --same-device rehearsal carrying the measured bucket plan (communicator probe),
# (b) optimiser placement under emulated 8-rank RCCL traffic (per-bucket Adam on the comm stream vs in
# step()), ViT-B/16 and ResNet-50 --force-comm
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step rehearsal4 600 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 4 --same-device --steps 5 --warmup 3
B="python bench.py --steps 20 --warmup 10 --force-comm"
for m in vit_b16 resnet50; do
  step emu_ov1_$m 300 0 $B --model $m --emulate-comm 64:300 --overlap-opt 1
  step emu_ov0_$m 300 0 $B --model $m --emulate-comm 64:300 --overlap-opt 0
  step emu_ov1b_$m 300 0 $B --model $m --emulate-comm 64:300 --overlap-opt 1
  step emu_ov0b_$m 300 0 $B --model $m --emulate-comm 64:300 --overlap-opt 0
done
echo done
