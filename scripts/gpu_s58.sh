#!/bin/bash
# session 58/62/66: full GPU suite, smoke, all three benchmark configs on the current tree
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 0 python bench.py
step bench_vit 300 0 python bench.py --model vit_b16
step bench_deq 300 0 python bench.py --model deq
echo done
