#!/bin/bash
# rd4ap: HIP-graph step (--graph) vs eager on the final tree, same box, interleaved; ResNet-50 and ViT-B/16
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step r50_plain_a 300 0 python -u bench.py --steps 20 --warmup 10
step r50_graph_a 300 0 python -u bench.py --steps 20 --warmup 10 --graph
step r50_plain_b 300 0 python -u bench.py --steps 20 --warmup 10
step r50_graph_b 300 0 python -u bench.py --steps 20 --warmup 10 --graph
step vit_plain_a 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_graph_a 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --graph
step vit_plain_b 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_graph_b 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --graph
echo done
