#!/bin/bash
# rd3zh: N=1 --force-comm tax vs the comm stream's priority (high, default, vs normal)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step r50 300 0 python bench.py --steps 20 --warmup 10
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_comm_p0 300 0 env FLUXMPI_COMM_PRIORITY=0 python bench.py --steps 20 --warmup 10 --force-comm
step r50b 300 0 python bench.py --steps 20 --warmup 10
step r50_commb 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_comm_p0b 300 0 env FLUXMPI_COMM_PRIORITY=0 python bench.py --steps 20 --warmup 10 --force-comm
echo done
