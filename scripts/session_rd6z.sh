#!/bin/bash
# round 6: ViT-B/16 plain Linear forwards with K <= 1024 (qkv, proj) on gemm_nt by default; fc2 stays
# on hipBLASLt. Tests, interleaved A/B against FLUXMPI_GEMM_NT_PLAIN_FWD_MAX_K=0, steady trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step tests 600 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py tests/test_vit_model_gpu.py tests/test_gemm_nt_gpu.py tests/test_vit_gpu.py
B="python bench.py --model vit_b16 --steps 20 --warmup 10"
for r in 1 2 3; do
  step vit_new_$r 300 0 $B
  step vit_old_$r 300 0 env FLUXMPI_GEMM_NT_PLAIN_FWD_MAX_K=0 $B
done
cd /tmp
step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd6z" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
