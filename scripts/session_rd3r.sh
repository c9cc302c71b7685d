#!/bin/bash
# rd3r: attention backward column-sum partials (packed QKV bias gradient without a colsum pass);
# DEQ profile; the --force-comm tax at the round-3 defaults (plain vs forced, profiles of both)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 300 1 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_linear_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_nocs 300 0 env FLUXMPI_ATTN_COLSUM=0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_nocsb 300 0 env FLUXMPI_ATTN_COLSUM=0 python bench.py --model vit_b16 --steps 20 --warmup 10
step r50 300 0 python bench.py --steps 20 --warmup 10
step r50_comm 300 0 python bench.py --steps 20 --warmup 10 --force-comm
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3r" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq_rd3r" -o run --output-format csv -- python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_r50_comm 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50comm_rd3r" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5 --force-comm; cd "$ROOT"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo done
