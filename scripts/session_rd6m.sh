#!/bin/bash
# round 6 final check: the whole GPU suite, smoke(), bench lines of the final tree (ResNet-50 headline, --force-comm,
# ViT-B/16, DEQ / DEQ-CIFAR with the converging presets and their 2-rank same-device rehearsals),
# steady-state kernel traces of ResNet-50 and DEQ-CIFAR
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 1000 0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 0 python -c "import __graft_entry__ as g; g.smoke()"
B="python bench.py --steps 20 --warmup 10"
step resnet 300 0 python bench.py
step resnet_b 300 0 $B
step resnet_comm 300 0 $B --force-comm
step vit 300 0 $B --model vit_b16
step deq 300 0 $B --model deq
step deq_cifar 300 0 $B --model deq_cifar --force-comm
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step deq_2rank 400 0 $R --master-port 29521 bench.py --gpus 2 --same-device --model deq --steps 10 --warmup 5
step deqc_2rank 400 0 $R --master-port 29522 bench.py --gpus 2 --same-device --model deq_cifar --steps 10 --warmup 5
cd /tmp
step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd6m" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 5
step prof_deqc 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deqc_rd6m" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq_cifar --force-comm --steps 5 --warmup 5
cd "$ROOT"
echo done
