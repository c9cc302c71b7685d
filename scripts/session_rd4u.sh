#!/bin/bash
# rd4u: bottleneck bn2 + ReLU folded into conv3's A load (FLUXMPI_BN2_FOLD=1) vs the separate bn2 pass,
# ResNet-50 interleaved, same tree; fused-block tests
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_fb 400 0 $T tests/test_fused_block_gpu.py -m gpu
FLUXMPI_BN2_FOLD=1 step r50_fold_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_base_1 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_BN2_FOLD=1 step r50_fold_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_base_2 300 0 python -u bench.py --steps 20 --warmup 10
echo done
