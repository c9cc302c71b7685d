# shared helpers for GPU sessions: `source scripts/gpu_lib.sh`
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
# step <name> <timeout_s> <allow_test_failure 0|1> cmd...
step() { local name=$1 t=$2 allow=$3; shift 3; echo "[$(date +%T)] $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  grep -h '"metric"' "$OUT/$name.log" >> "$OUT/bench_results.jsonl" 2>/dev/null
  if [ $rc -ne 0 ]; then if [ "$allow" = "1" ] && [ $rc -eq 1 ]; then return 0; fi; exit $rc; fi; }
build_ext() { step build 300 0 python -c "import fluxmpi_amd._build as b; print(b.build())"; }
