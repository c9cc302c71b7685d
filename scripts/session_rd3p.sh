#!/bin/bash
# rd3p: in-kernel BatchNorm finalize without per-workgroup L2 write-back; two-phase attention backward
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_bn 300 1 python -u -m pytest tests/test_batchnorm.py tests/test_fused_block_gpu.py tests/test_resnet_ops_gpu.py tests/test_vit_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step r50_fin1 300 0 python bench.py --steps 20 --warmup 10
step r50_fin0 300 0 env FLUXMPI_BN_FIN=0 python bench.py --steps 20 --warmup 10
step r50_fin1b 300 0 python bench.py --steps 20 --warmup 10
step r50_fin0b 300 0 env FLUXMPI_BN_FIN=0 python bench.py --steps 20 --warmup 10
step vit_pair 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_two 300 0 env FLUXMPI_ATTN_BWD=two python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_pairb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_twob 300 0 env FLUXMPI_ATTN_BWD=two python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd3p" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_vit_two 300 0 env FLUXMPI_ATTN_BWD=two rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_two_rd3p" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo done
