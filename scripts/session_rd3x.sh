#!/bin/bash
# rd3x: tanh-form GELU (NNlib's gelu) with fc1 on hipBLASLt's bias + GELU epilogue
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gelu 400 1 python -u -m pytest tests/test_gelu.py tests/test_gemm256_gpu.py tests/test_linear_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_erf 300 1 env FLUXMPI_GELU=erf python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_noblt 300 1 env FLUXMPI_GELU_BLASLT=0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_erfb 300 1 env FLUXMPI_GELU=erf python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_tune 300 1 env FLUXMPI_BLASLT_TUNE=1 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp
step prof_vit 300 1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3x" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
