#!/bin/bash
# rd4ao: DDP-path tax on the final tree, same box: plain vs --force-comm vs --force-comm + emulated RCCL
# CU footprint (64 WG x 300 us per bucket), ResNet-50 and ViT-B/16; functional-API DEQ-CIFAR line
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step r50_plain 300 0 python -u bench.py --steps 20 --warmup 10
step r50_fc 300 0 python -u bench.py --steps 20 --warmup 10 --force-comm
step r50_emu 300 0 python -u bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step vit_plain 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_fc 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
step vit_emu 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm --emulate-comm 64:300
step deqc_func 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5 --api functional --force-comm
echo done
