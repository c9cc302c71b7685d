#!/bin/bash
# session 31: kernel trace of the BatchNorm op microbenchmark (per-kernel durations by shape)
source "$(dirname "$0")/gpu_lib.sh"
cd /tmp && step prof_bn 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bn" -o run --output-format csv -- python3 "$ROOT/scripts/bench_bn_ops.py"
echo done
