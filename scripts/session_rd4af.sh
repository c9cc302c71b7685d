#!/bin/bash
# rd4af: L2 hit rate and wave-state counters of every ResNet-50 kernel (one short bench run per pass)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp
step pmc_r50 400 0 timeout -s KILL 360 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
  -d "$OUT/pmc_r50" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 2
cd "$ROOT"
echo done
