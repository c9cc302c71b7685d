#!/bin/bash
# rd3t: PMC counters of the attention kernels at the ViT-B/16 shape (two passes, 8 SQ counters each)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
cd /tmp
step pmc_a 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/pmc_attn_a" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_attn.py"
step pmc_b 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/pmc_attn_b" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_attn.py"
cd "$ROOT"
echo done
