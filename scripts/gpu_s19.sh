#!/bin/bash
# session 19: HIP-graph step and conv=fused vs the hybrid default; DEQ at 28x28; profile
source "$(dirname "$0")/gpu_lib.sh"
step bench_graph 400 0 python bench.py --graph
step bench_fused 400 0 python bench.py --conv fused
step bench_fused_graph 400 0 python bench.py --conv fused --graph
step bench_deq 300 0 python bench.py --model deq --steps 10 --warmup 5
cd /tmp && step prof19 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof19" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
