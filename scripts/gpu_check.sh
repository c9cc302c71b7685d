#!/bin/bash
# One GPU-box session: tests, smoke, bench variants, rocprof kernel stats.
# Every GPU step has its own time limit. A test *failure* (exit 1) lets the
# session continue; a crash, abort, fault or timeout (any other non-zero
# status) ends it immediately (no retries).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <allow_fail:0|1> cmd...
  local name=$1 t=$2 allow=$3; shift 3
  echo "[$(date +%T)] $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then
    if [ "$allow" = "1" ] && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}

STEPS="${STEPS:-build pytest smoke bench prof}"
for s in $STEPS; do
  case $s in
    build) step build 300 0 python -c "import fluxmpi_amd._build as b; print(b.build())" ;;
    pytest) step pytest_gpu 360 1 python -m pytest tests -m gpu -q ;;
    smoke) step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_gemm 300 0 python bench.py --steps 20 --warmup 10
           step bench_miopen 300 0 python bench.py --steps 20 --warmup 10 --conv miopen ;;
    prof) cd /tmp && step prof 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 3; cd "$ROOT" ;;
    *) echo "unknown step $s" ;;
  esac
done
echo done
