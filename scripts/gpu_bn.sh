#!/bin/bash
# GPU session 2: fused-BN tests + bench matrix (conv x norm) + profile of the best config.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { local name=$1 t=$2 allow=$3; shift 3; echo "[$(date +%T)] $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then if [ "$allow" = "1" ] && [ $rc -eq 1 ]; then return 0; fi; exit $rc; fi; }
step build 300 0 python -c "import fluxmpi_amd._build as b; print(b.build())"
step pytest_gpu 400 1 python -m pytest tests -m gpu -q -x
step bench_miopen_fused 300 0 python bench.py --steps 20 --warmup 10 --conv miopen --norm fused
step bench_gemm_fused 300 0 python bench.py --steps 20 --warmup 10 --conv gemm --norm fused
step bench_miopen_torch 300 0 python bench.py --steps 20 --warmup 10 --conv miopen --norm torch
cd /tmp && step prof 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof2" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --conv miopen --norm fused
echo done
