#!/bin/bash
# rd4r: conv routing fixes — the 3x3 forward's autotune / engine 0 reaches gemm_nt, the model's 1x1
# forwards take gemm_nt where qualified — vs the committed routing (ab/), ResNet-50 interleaved; conv tests
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_conv 400 0 $T tests/test_conv_gpu.py tests/test_resnet_ops_gpu.py tests/test_fused_block_gpu.py -m gpu
step r50_new_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_1 300 0 python -u ab/bench.py --steps 20 --warmup 10
step r50_new_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_2 300 0 python -u ab/bench.py --steps 20 --warmup 10
echo done
