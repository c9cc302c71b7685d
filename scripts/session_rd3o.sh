#!/bin/bash
# rd3o: in-kernel BatchNorm finalize + direct gradient delivery — GPU suite, smoke, same-box A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step r50_fin1 300 0 python bench.py --steps 20 --warmup 10
step r50_fin0 300 0 env FLUXMPI_BN_FIN=0 python bench.py --steps 20 --warmup 10
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_comm_nodirect 300 0 env FLUXMPI_DIRECT_GRADS=0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_emu 300 0 python bench.py --steps 20 --warmup 10 --force-comm --emulate-comm 64:300
step r50_fin1b 300 0 python bench.py --steps 20 --warmup 10
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step deq 300 0 python bench.py --model deq --steps 20 --warmup 10
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd3o" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_r50_comm 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50comm_rd3o" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5 --force-comm; cd "$ROOT"
echo done
