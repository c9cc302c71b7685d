#!/bin/bash
# session 39: HIP-graph capture of the full ResNet-50 step (bench --graph) vs eager
source "$(dirname "$0")/gpu_lib.sh"
step bench_graph 500 0 python bench.py --graph
step bench_eager 400 0 python bench.py
echo done
