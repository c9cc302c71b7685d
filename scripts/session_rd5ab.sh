#!/bin/bash
# round 5: RCCL CU-footprint emulation at N = 1 (bench --force-comm --emulate-comm WGS:GBPS[:THREADS[:LDS_KB]]):
# how much the current kernels (persistent / one-round grids included) lose when comm workgroups hold CUs
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10 --force-comm"
step comm 300 0 $B
step emu32 300 0 $B --emulate-comm 32:300:256
step emu64 300 0 $B --emulate-comm 64:150:512:32
step emu64_r2 300 0 env FLUXMPI_GRID_ROUNDS=2 $B --emulate-comm 64:150:512:32
step comm_b 300 0 $B
step vit_comm 300 0 $B --model vit_b16
step vit_emu64 300 0 $B --model vit_b16 --emulate-comm 64:150:512:32
echo done
