#!/bin/bash
# round 5: software-pipelined gemm_wgrad (split-K weight gradient): numerics, same-box A/B vs the
# previous kernel over the ResNet-50 weight-gradient shapes, ResNet-50
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_wg 600 1 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_wgrad3x3n_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step wg_new 300 0 python scripts/bench_wgrad_resnet.py
step wg_old 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_wg_old.so python scripts/bench_wgrad_resnet.py
step resnet 300 0 $B
step resnet_old 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_wg_old.so python scripts/diag/bench_variant.py --steps 20 --warmup 10
step resnet_b 300 0 $B
echo done
