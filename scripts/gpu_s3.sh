#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_bn 300 1 python -m pytest tests/test_batchnorm.py -m gpu -q -x
step b256 300 0 python bench.py --steps 20 --warmup 10
step b256_find 600 0 python bench.py --steps 20 --warmup 10 --miopen-find 1
step b128 300 0 python bench.py --steps 20 --warmup 10 --batch 128
step b384 300 0 python bench.py --steps 20 --warmup 10 --batch 384
cd /tmp && step prof3 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 3
echo done
