#!/bin/bash
# rd3zd: bucket fence without the system-scope release (comm/fence.cpp) vs torch's wait_stream, --force-comm
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_comm 400 1 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step r50 300 0 python bench.py --steps 20 --warmup 10
step r50_fence 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_torch 300 0 env FLUXMPI_NATIVE_FENCE=0 python bench.py --steps 20 --warmup 10 --force-comm
step r50b 300 0 python bench.py --steps 20 --warmup 10
step r50_fenceb 300 0 python bench.py --steps 20 --warmup 10 --force-comm
step r50_torchb 300 0 env FLUXMPI_NATIVE_FENCE=0 python bench.py --steps 20 --warmup 10 --force-comm
echo done
