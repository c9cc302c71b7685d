#!/bin/bash
# rd3zj: confirmation of the normal-priority comm stream default: comm / DDP GPU tests, plain vs --force-comm
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_comm 400 1 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step r50 300 0 python bench.py
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50b 300 0 python bench.py --steps 20 --warmup 10
step r50_commb 300 0 python bench.py --steps 20 --warmup 10 --force-comm
echo done
