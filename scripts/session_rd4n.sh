#!/bin/bash
# rd4n: same-box A/B of the gelu'(h) epilogue (this tree) vs the committed tree (ab/: the h epilogue), ViT-B/16
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step vit_deriv_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_main_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step vit_deriv_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_main_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
echo done
