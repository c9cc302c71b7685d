#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_bn 300 1 python -m pytest tests/test_batchnorm.py -m gpu -q -x
step bench_default 400 0 python bench.py
step bench_stem 500 0 python scripts/bench_stem.py
step bench_vit 500 0 python bench.py --model vit_b16 --steps 10 --warmup 5
step bench_deq 500 0 python bench.py --model deq --image 28 --steps 10 --warmup 5
echo done
