#!/bin/bash
# round 6: ViT-B/16 --force-comm steady trace of the final tree
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
step prof_vitc 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vitc_rd6am" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5 --force-comm
cd "$ROOT"
echo done
