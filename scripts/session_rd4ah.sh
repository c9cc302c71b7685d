#!/bin/bash
# rd4ah: final validation of the round-4 tree — full GPU suite, smoke(), default bench, ViT, DDP-path lines
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step gpu_suite 900 0 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 0 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 600 0 python -u bench.py
step vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step r50_force_comm 300 0 python -u bench.py --steps 20 --warmup 10 --force-comm
step vit_force_comm 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
step deq 400 0 python -u bench.py --model deq --steps 10 --warmup 5
step deqc 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5 --force-comm
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd4ah" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd4ah" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
echo done
