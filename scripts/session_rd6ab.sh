#!/bin/bash
# round 6 final check of the final tree: whole GPU suite, smoke(), bench lines, ResNet-50 steady trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 1000 0 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 0 python -c "import __graft_entry__ as g; g.smoke()"
B="python bench.py --steps 20 --warmup 10"
step resnet 300 0 python bench.py
step resnet_comm 300 0 $B --force-comm
step vit 300 0 $B --model vit_b16
step vit_comm 300 0 $B --model vit_b16 --force-comm
step deq 300 0 $B --model deq
step deq_cifar 300 0 $B --model deq_cifar
cd /tmp
step prof_resnet 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_resnet_rd6ab" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd "$ROOT"
echo done
