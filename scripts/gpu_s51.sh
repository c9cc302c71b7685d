#!/bin/bash
# session 51: attention backward micro-bench + PMC counters of our two kernels
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step battn 120 0 python scripts/bench_attn.py
cd /tmp
step pmc1 60 0 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d "$OUT/pmc1" -o run --output-format csv -- python3 "$ROOT/scripts/bench_attn.py"
step pmc2 60 0 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc2" -o run --output-format csv -- python3 "$ROOT/scripts/bench_attn.py"
echo done
