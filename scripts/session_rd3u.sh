#!/bin/bash
# rd3u: conflict-free attention image swizzle (row & 6) — tests, ViT bench, PMC pass, profile
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 300 1 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp
step pmc_a 90 0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/pmc_attn_a_rd3u" -o run \
  --output-format csv -- python3 "$ROOT/scripts/pmc_attn.py"
step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3u" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
# LDS bank-conflict survey of every kernel of a short ResNet-50 and ViT-B/16 run
cd /tmp
step pmc_lds_r50 240 0 timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc_lds_r50_rd3u" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 2 --choices shipped
step pmc_lds_vit 240 0 timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc_lds_vit_rd3u" -o run \
  --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 2 --warmup 2
cd "$ROOT"
echo done2
