#!/bin/bash
# session 30: BatchNorm kernel bandwidth per ResNet-50 shape
source "$(dirname "$0")/gpu_lib.sh"
step bench_bn_ops 300 0 python scripts/bench_bn_ops.py
echo done
