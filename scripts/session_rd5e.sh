#!/bin/bash
# round 5: split-K tail off by default, DEQ solver tolerances above the bf16 floor — residual
# trajectories, A/B benches, steady-state profiles, the GPU suite and the 2-rank rehearsal
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
prof() {  # prof <name> <bench args...>
  local name=$1; shift
  cd /tmp && step "prof_${name}" 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${name}_rd5e" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" "$@"; cd "$ROOT"
}
step resid_mnist 240 0 python scripts/diag/deq_residual.py --model deq
step resid_cifar 240 0 python scripts/diag/deq_residual.py --model deq_cifar --iters 10,20,30,45,60
step resnet 300 0 $B
step resnet_s8 300 0 env FLUXMPI_GEMM_NT_SPLIT=8 $B
step vit 300 0 $B --model vit_b16
step vit_s8 300 0 env FLUXMPI_GEMM_NT_SPLIT=8 $B --model vit_b16
step deq 300 0 $B --model deq
step deq_tol4 300 0 $B --model deq --deq-solver tol=1e-4,bwd_tol=1e-4
step deq_cifar 300 0 $B --model deq_cifar --force-comm
prof resnet50 --steps 5 --warmup 5
prof vit --model vit_b16 --steps 5 --warmup 5 --force-comm --overlap-opt 1
prof deq_cifar --model deq_cifar --steps 5 --warmup 5 --force-comm
step smoke 240 0 python -c "import __graft_entry__ as g; g.smoke()"
step bench_2rank 300 0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 3 --batch 32 --same-device
echo done
