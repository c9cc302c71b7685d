#!/bin/bash
# round 5: DEQ solver graphs without per-iteration scalar / iterate copies (residual written into the
# replay buffer, the chunk's last adjoint iterate into the static u, amin / amax with out=):
# GPU tests, same-box A/B against the previous Python package (exp/olddeq), kernel trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_deq 600 1 python -u -m pytest tests/test_deq.py -m gpu -x -q --timeout 120 --timeout-method thread
for r in a b; do
step d_new_$r 300 0 python bench.py --model deq --steps 20 --warmup 10
step d_old_$r 300 0 python exp/olddeq/bench.py --model deq --steps 20 --warmup 10
done
step dc_new 300 0 python bench.py --model deq_cifar --steps 20 --warmup 10 --force-comm
step dc_old 300 0 python exp/olddeq/bench.py --model deq_cifar --steps 20 --warmup 10 --force-comm
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_rd5af" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5; cd "$ROOT"
echo done
