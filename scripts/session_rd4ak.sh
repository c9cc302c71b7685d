#!/bin/bash
# rd4ak: BatchNorm apply / dx passes with 4 vectors per lane per iteration (FLUXMPI_BN_UNROLL=4) vs 2,
# ResNet-50 interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
FLUXMPI_BN_UNROLL=4 step r50_u4_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_u2_1 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_BN_UNROLL=4 step r50_u4_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_u2_2 300 0 python -u bench.py --steps 20 --warmup 10
echo done
