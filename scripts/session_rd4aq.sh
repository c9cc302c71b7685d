#!/bin/bash
# rd4aq: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs default, same box, interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step r50_def_a 300 0 python -u bench.py --steps 20 --warmup 10
step r50_ka_a 300 0 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --steps 20 --warmup 10
step r50_def_b 300 0 python -u bench.py --steps 20 --warmup 10
step r50_ka_b 300 0 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --steps 20 --warmup 10
step vit_def_a 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_ka_a 300 0 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --model vit_b16 --steps 10 --warmup 5
echo done
