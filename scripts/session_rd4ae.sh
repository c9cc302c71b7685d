#!/bin/bash
# rd4ae: PMC counters of the ViT weight gradients (wgrad256 + split-K reduce): wave states, MFMA busy,
# LDS conflicts, L2 hits, beyond-L2 bytes
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp
step pmc_a 120 0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/pmc_wg_a" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_wgrad.py"
step pmc_b 120 0 timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 TCC_HIT_sum TCC_MISS_sum \
  -d "$OUT/pmc_wg_b" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_wgrad.py"
step pmc_c 120 0 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_wg_c" -o run --output-format csv \
  -- python3 "$ROOT/scripts/pmc_wgrad.py"
step trace 120 0 timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/pmc_wg_t" -o run --output-format csv \
  -- python3 "$ROOT/scripts/pmc_wgrad.py"
cd "$ROOT"
echo done
