#!/bin/bash
# session 47 (fresh container rebuild): full GPU suite, smoke, default bench, kernel stats
source "$(dirname "$0")/gpu_lib.sh"
step pytest_all 900 0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 0 python bench.py
cd /tmp && step prof47 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof47" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
