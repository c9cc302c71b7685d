#!/bin/bash
# rd4z: bn3-only BN-backward link that leaves the downsample blocks' dual BatchNorm in place
# (FLUXMPI_BN_LINK=bn3) vs none, ResNet-50 interleaved; tests
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_fb 400 0 $T tests/test_fused_block_gpu.py -m gpu
FLUXMPI_BN_LINK=bn3 step r50_bn3_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_base_1 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_BN_LINK=bn3 step r50_bn3_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_base_2 300 0 python -u bench.py --steps 20 --warmup 10
echo done
