#!/bin/bash
# round 5: GroupNorm with up to 1024 lanes per sample (was 256) — DEQ GPU tests, same-box A/B on
# DEQ-CIFAR against a GN_THREADS=256 variant build
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="--model deq_cifar --force-comm --steps 20 --warmup 10"
step pytest_deq 600 0 python -u -m pytest tests/test_deq.py -m gpu -x -q --timeout 120 --timeout-method thread
step cifar_gn256 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn256.so python scripts/diag/bench_variant.py $B
step cifar_gn1024 300 0 python bench.py $B
step cifar_gn256_b 300 0 env FLUXMPI_C_VARIANT=exp/variants/_C_gn256.so python scripts/diag/bench_variant.py $B
step cifar_gn1024_b 300 0 python bench.py $B
cd /tmp && step prof_deq_cifar 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_cifar_rd5j" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5 --force-comm; cd "$ROOT"
echo done
