#!/bin/bash
# round 6: the fused DEQ cell kernels at 16 waves per sample (FLUXMPI_DEQ_CELL_FWD_WAVES /
# FLUXMPI_DEQ_CELL_VJP_WAVES) vs 8: numerics tests per variant, kernel micro-benchmark, MNIST lines
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py"
step test_w8 300 0 $T
step test_w16 300 0 env FLUXMPI_DEQ_CELL_FWD_WAVES=16 FLUXMPI_DEQ_CELL_VJP_WAVES=16 $T
for r in 1 2; do
  step mb_w8_$r 120 0 python scripts/bench_deq_cell.py
  step mb_w16_$r 120 0 env FLUXMPI_DEQ_CELL_FWD_WAVES=16 FLUXMPI_DEQ_CELL_VJP_WAVES=16 python scripts/bench_deq_cell.py
done
B="python bench.py --model deq --steps 40 --warmup 10"
step deq_w8 300 0 $B
step deq_f16 300 0 env FLUXMPI_DEQ_CELL_FWD_WAVES=16 $B
step deq_w8b 300 0 $B
step deq_f16b 300 0 env FLUXMPI_DEQ_CELL_FWD_WAVES=16 $B
echo done
