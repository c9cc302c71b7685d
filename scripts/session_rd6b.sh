#!/bin/bash
# round 6: conv_c3 stem kernels (GPU tests), DEQ contraction diagnostics (which parameters drift
# under training, and whether a max-norm projection keeps the solves converging), DEQ benches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step test_c3 300 0 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_c3_gpu.py tests/test_ddp_gpu.py
for c in none conv conv+gn; do
  step diag_deq_$c 200 0 env FLUXMPI_DEQ_CONSTRAIN=$c python scripts/diag_deq_contract.py --model deq --steps 40
  step diag_deqc_$c 300 0 env FLUXMPI_DEQ_CONSTRAIN=$c python scripts/diag_deq_contract.py --model deq_cifar --steps 40
done
B="python bench.py --steps 20 --warmup 10"
step deq_cifar 300 0 $B --model deq_cifar --force-comm
cd /tmp
step prof_deqc 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deqc_rd6b" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5 --force-comm
cd "$ROOT"
echo done
