#!/bin/bash
# rd4ar: end-of-session check of the committed tree with the .so from build(): GPU suite, smoke(), default bench
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step gpu_suite 900 0 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 0 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 0 python -u bench.py
echo done
