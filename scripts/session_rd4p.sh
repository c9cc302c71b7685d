#!/bin/bash
# rd4p: gemm_nt epilogue-store experiment (exp/: stores skipped / non-temporal / write-through)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step nt_exp 300 0 python -u exp/nt_exp.py
echo done
