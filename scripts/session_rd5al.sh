#!/bin/bash
# round 5: conv3x3n counters (stage-2 and stage-1 shapes): kernel trace, wave states / LDS, instruction mix, HBM bytes
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step trace 120 0 timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/c3n_trace" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
step pmc_a 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/c3n_pmc_a" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
step pmc_b 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/c3n_pmc_b" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
step pmc_c 90 0 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c3n_pmc_c" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
step pmc_d 90 0 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c3n_pmc_d" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
export SHAPE=256,64,56,56
step pmc_a64 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/c3n_pmc_a64" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_c3n.py"
echo done
