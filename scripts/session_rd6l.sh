#!/bin/bash
# round 6 final check, part 1: the whole GPU suite and smoke() on the final tree
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 1000 0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 0 python -c "import __graft_entry__ as g; g.smoke()"
echo done
