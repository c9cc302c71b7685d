#!/bin/bash
# rd3zc: final round-3 validation of the committed tree: full GPU suite, smoke, headline bench, ViT
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step r50 300 0 python bench.py
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step deq 300 0 python bench.py --model deq --steps 20 --warmup 10
echo done
