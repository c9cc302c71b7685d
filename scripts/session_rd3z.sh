#!/bin/bash
# rd3z: validation of the round-3 defaults (pipelined <13> attention, tanh GELU): full GPU suite, smoke, benches, profiles
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step r50 300 0 python bench.py
step r50b 300 0 python bench.py --steps 20 --warmup 10
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step bench_2rank 300 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 3 --batch 32 --same-device
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step deq 300 0 python bench.py --model deq --steps 20 --warmup 10
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd3z" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
step vit_erf 300 0 env FLUXMPI_GELU=erf python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3z" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
