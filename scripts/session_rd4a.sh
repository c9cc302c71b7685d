#!/bin/bash
# rd4b: persistent gemm_nt of gemm_nt.hip (ping-pong 256x256 NT GEMM) vs hipBLASLt and gemm256
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
echo done
