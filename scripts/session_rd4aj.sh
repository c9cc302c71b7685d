#!/bin/bash
# rd4aj: attention kernels' L2 hit rate and wave states (ViT-B/16 shape)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp
step pmc_attn 120 0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_attn_l2" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_attn.py"
step pmc_attn_f 120 0 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_attn_fetch" -o run --output-format csv \
  -- python3 "$ROOT/scripts/pmc_attn.py"
cd "$ROOT"
echo done
