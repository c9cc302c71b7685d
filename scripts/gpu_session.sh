#!/bin/bash
# One GPU-box session, parametrised by STEPS (space-separated) and TAG (output-name suffix):
#
#   STEPS="smoke bench bench_vit prof" TAG=s3 bash scripts/gpu_session.sh
#
# Every GPU step runs under its own `timeout -k 10`; a test *failure* (exit 1) of a step
# marked allow=1 lets the session continue, any other non-zero status (crash, abort, fault,
# time limit) ends it at once, with no retries. Bench JSON lines are collected in
# gpurun_out/bench_results.jsonl; rocprofv3 output goes to gpurun_out/prof_<what>_<TAG>/.
source "$(dirname "$0")/gpu_lib.sh"
TAG="${TAG:-x}"
STEPS="${STEPS:-smoke bench}"
BENCH_STEPS="${BENCH_STEPS:-20}"
BENCH_WARMUP="${BENCH_WARMUP:-10}"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"

prof() {  # prof <name> <bench args...>: kernel trace + stats of a short bench run
  local name=$1; shift
  cd /tmp && step "prof_${name}" 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${name}_${TAG}" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" "$@"; cd "$ROOT"
}

for s in $STEPS; do
  case $s in
    build) build_ext ;;
    pytest) step pytest_gpu 900 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytest_comm) step pytest_comm 300 1 python -u -m pytest tests/test_comm_gpu.py -m gpu -x -v --timeout 120 \
                   --timeout-method thread ;;
    pytest_gemm) step pytest_gemm 600 1 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv_gpu.py \
                   tests/test_gemm_nt_gpu.py tests/test_fused_block_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytest_vit) step pytest_vit 600 1 python -u -m pytest tests/test_vit_model_gpu.py tests/test_vit_gpu.py tests/test_linear_gpu.py \
                   tests/test_gelu.py tests/test_layernorm.py -m gpu -x -q -s --timeout 300 --timeout-method thread ;;
    pytest_nt) step pytest_nt 600 1 python -u -m pytest tests/test_gemm_nt_gpu.py -m gpu -x -v --timeout 120 \
                 --timeout-method thread ;;
    bench_nt) step bench_nt 600 0 python scripts/bench_gemm_nt.py ;;
    bench_vit_all) step bench_vit_all 300 0 env FLUXMPI_GEMM_NT=all python bench.py --model vit_b16 --steps "$BENCH_STEPS" \
                     --warmup "$BENCH_WARMUP" ;;
    bench_vit_nosplit) step bench_vit_nosplit 300 0 env FLUXMPI_GEMM_NT_SPLIT=0 python bench.py --model vit_b16 \
                         --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" ;;
    bench_nosplit) step bench_nosplit 300 0 env FLUXMPI_GEMM_NT_SPLIT=0 python bench.py --steps "$BENCH_STEPS" \
                     --warmup "$BENCH_WARMUP" ;;
    smoke) step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 0 python bench.py --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" ;;
    bench_graph) step bench_graph 300 0 python bench.py --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" --graph ;;
    bench_comm) step bench_comm 300 0 python bench.py --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" --force-comm ;;
    bench_graph_comm) step bench_graph_comm 300 0 python bench.py --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" \
                        --graph --force-comm ;;
    bench_vit) step bench_vit 300 0 python bench.py --model vit_b16 --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" ;;
    bench_vit_comm) step bench_vit_comm 300 0 python bench.py --model vit_b16 --steps "$BENCH_STEPS" \
                      --warmup "$BENCH_WARMUP" --force-comm ;;
    bench_deq) step bench_deq 300 0 python bench.py --model deq --steps "$BENCH_STEPS" --warmup "$BENCH_WARMUP" ;;
    bench_2rank) step bench_2rank 300 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                   --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 3 \
                   --batch 32 --same-device ;;
    probe2) step probe2 120 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
              --master-addr 127.0.0.1 --master-port 29521 scripts/probe_two_ranks_one_gpu.py ;;
    vit_gemm) step vit_gemm 300 0 python scripts/bench_vit_gemm.py ;;
    prof) prof resnet50 --steps 5 --warmup 5 ;;
    prof_comm) prof resnet50_comm --steps 5 --warmup 5 --force-comm ;;
    prof_vit) prof vit --model vit_b16 --steps 5 --warmup 5 ;;
    prof_deq) prof deq --model deq --steps 5 --warmup 5 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
