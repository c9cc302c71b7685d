#!/bin/bash
# rd3za: HIP GELU forward (gelu.hip gelu_fwd) vs PyTorch's elementwise GELU in ViT-B/16
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gelu 400 1 python -u -m pytest tests/test_gelu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_torch 300 1 env FLUXMPI_GELU_FWD=torch python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_torchb 300 1 env FLUXMPI_GELU_FWD=torch python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp && step prof_vit 300 1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3za" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
