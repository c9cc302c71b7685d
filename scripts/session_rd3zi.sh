#!/bin/bash
# rd3zi: comm stream priority with an emulated RCCL CU footprint (does normal priority delay the comm?)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step emu_hi 300 0 python bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step emu_p0 300 0 env FLUXMPI_COMM_PRIORITY=0 python bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step emu_hib 300 0 python bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step emu_p0b 300 0 env FLUXMPI_COMM_PRIORITY=0 python bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step plain 300 0 python bench.py --steps 20 --warmup 10
echo done
