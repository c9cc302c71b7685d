#!/bin/bash
# round 6: wave-specialised stem backward (tests vs fp32, kernel time vs the row-pair kernel,
# ResNet-50 A/B); DEQ solver presets that end by tolerance (MNIST tolerance sweep, 2-rank rehearsal)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_stem 300 0 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem_gpu.py
step stem_ws 120 0 python scripts/bench_stem_bwd.py
step stem_pair 120 0 env FLUXMPI_STEM_BWD=pair python scripts/bench_stem_bwd.py
step stem_ws_b 120 0 python scripts/bench_stem_bwd.py
step stem_pair_b 120 0 env FLUXMPI_STEM_BWD=pair python scripts/bench_stem_bwd.py
B="python bench.py --steps 20 --warmup 10"
step r50_ws 300 0 $B
step r50_pair 300 0 env FLUXMPI_STEM_BWD=pair $B
step r50_ws_b 300 0 $B
step r50_pair_b 300 0 env FLUXMPI_STEM_BWD=pair $B
step deq_t1b2 300 0 $B --model deq --deq-solver max_iter=60,tol=1e-2,bwd_iter=60,bwd_tol=2e-2
step deq_t2b2 300 0 $B --model deq --deq-solver max_iter=60,tol=2e-2,bwd_iter=60,bwd_tol=2e-2
step deqc_c 300 0 $B --model deq_cifar --deq-solver max_iter=60,tol=2e-2,bwd_iter=60,bwd_tol=1e-2
echo done
