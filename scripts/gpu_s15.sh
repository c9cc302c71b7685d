#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q -x
step bench_default 500 0 python bench.py
step vit_tune 700 0 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME="$OUT/tunableop_vit.csv" PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10 PYTORCH_TUNABLEOP_MAX_WARMUP_ITERATIONS=2 python bench.py --model vit_b16 --steps 5 --warmup 2
ls "$OUT"/tunableop* || true
F=$(ls "$OUT"/tunableop_vit*.csv | head -1)
step vit_tuned 400 0 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME="$F" python bench.py --model vit_b16 --steps 10 --warmup 3
cd /tmp && step prof15 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof15" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
