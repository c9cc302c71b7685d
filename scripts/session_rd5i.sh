#!/bin/bash
# round 5: bf16 Anderson F history + gemm_nt residual epilogue (EPI 4) — DEQ / gemm_nt GPU tests,
# same-box A/B (fp32 history vs bf16)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="--steps 20 --warmup 10"
step pytest_deq 600 0 python -u -m pytest tests/test_deq.py tests/test_gemm_nt_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread
step deq_f32 300 0 python scripts/diag/bench_deq_f32hist.py --model deq $B
step deq_bf16 300 0 python bench.py --model deq $B
step cifar_f32 300 0 python scripts/diag/bench_deq_f32hist.py --model deq_cifar --force-comm $B
step cifar_bf16 300 0 python bench.py --model deq_cifar --force-comm $B
step deq_f32_b 300 0 python scripts/diag/bench_deq_f32hist.py --model deq $B
step deq_bf16_b 300 0 python bench.py --model deq $B
cd /tmp && step prof_deq_cifar 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_cifar_rd5i" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5 --force-comm; cd "$ROOT"
echo done
