#!/bin/bash
# rd4al: BatchNorm backward reduce passes with 2 rows in flight per lane (97-111 / 158 VGPRs instead of
# 138-140 / 240: four / three waves per SIMD) vs committed (ab/), ResNet-50 interleaved; BN tests
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_bn 400 0 $T tests/test_batchnorm.py tests/test_fused_block_gpu.py -m gpu
step r50_new_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_1 300 0 python -u ab/bench.py --steps 20 --warmup 10
step r50_new_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_2 300 0 python -u ab/bench.py --steps 20 --warmup 10
echo done
