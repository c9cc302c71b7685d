#!/bin/bash
# rd3zg: does the N=1 --force-comm tax scale with the bucket count? (7 buckets default vs 1-2 / ~25)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step r50 300 0 python bench.py --steps 20 --warmup 10
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_comm_big 300 0 env FLUXMPI_BUCKET_MB=256 FLUXMPI_FIRST_BUCKET_MB=256 FLUXMPI_TAIL_BUCKET_MB=0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_comm_small 300 0 env FLUXMPI_BUCKET_MB=2 FLUXMPI_FIRST_BUCKET_MB=2 python bench.py --steps 20 --warmup 10 --force-comm
step r50b 300 0 python bench.py --steps 20 --warmup 10
step r50_commb 300 0 python bench.py --steps 20 --warmup 10 --force-comm
echo done
