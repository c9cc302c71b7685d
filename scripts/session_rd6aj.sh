#!/bin/bash
# round 6 closing check of the final tree: whole GPU suite, smoke(), headline bench lines
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 1000 0 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 0 python -c "import __graft_entry__ as g; g.smoke()"
step resnet 300 0 python bench.py
step resnet_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step deq 300 0 python bench.py --model deq --steps 20 --warmup 10
step deq_cifar 300 0 python bench.py --model deq_cifar --steps 20 --warmup 10
echo done
