#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q -x
step bench_default 400 0 python bench.py
step bench_graph 400 0 python bench.py --graph
step smoke 300 0 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && step prof12 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof12" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
