#!/bin/bash
# rd3v: attention kernels with a compile-time tile count (T = 197) + software-pipelined forward
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 300 1 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_gen 300 0 env FLUXMPI_ATTN_GENERIC=1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_genb 300 0 env FLUXMPI_ATTN_GENERIC=1 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp
step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3v" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
step pmc_a 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/pmc_attn_a_rd3v" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_attn.py"
cd "$ROOT"
echo done
