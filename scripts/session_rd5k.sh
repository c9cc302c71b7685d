#!/bin/bash
# round 5: GroupNorm with up to 1024 lanes per sample (A/B against a GN_THREADS=256 variant build on
# DEQ-CIFAR) and the narrow-K 1x1 forward (conv1x1n: GPU tests, kernel table, ResNet-50 A/B)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
C="--model deq_cifar --force-comm --steps 20 --warmup 10"
B="--steps 20 --warmup 10"
step pytest 600 0 python -u -m pytest tests/test_deq.py tests/test_conv1x1n_gpu.py tests/test_conv3x3n_gpu.py tests/test_fused_block_gpu.py -m gpu \
  -x -q --timeout 120 --timeout-method thread
step bench_c1 240 0 python scripts/bench_conv1x1n.py
step bench_c3 240 0 python scripts/bench_conv3x3n.py
step cifar_gn256 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn256.so python scripts/diag/bench_variant.py $C
step cifar_gn1024 300 0 python bench.py $C
step r50_off 300 0 python scripts/diag/bench_no_conv1x1n.py $B
step r50_on 300 0 python bench.py $B
step cifar_gn256_b 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn256.so python scripts/diag/bench_variant.py $C
step cifar_gn1024_b 300 0 python bench.py $C
step r50_off_b 300 0 python scripts/diag/bench_no_conv1x1n.py $B
step r50_on_b 300 0 python bench.py $B
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd5k" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
echo done
