#!/bin/bash
# round 6: linbwd tests, DEQ Jacobian regularisation under training, ViT A/Bs (linbwd with the
# measured split choice; plain Linear forwards on gemm_nt), stem backward phase split
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_lb 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linbwd_gpu.py
for m in 0 1 2 3; do step stem_diag$m 120 0 env FLUXMPI_STEM_BWD_DIAG=$m python scripts/bench_stem_bwd.py; done
B="python bench.py --steps 20 --warmup 10 --model vit_b16"
step vit_a 300 0 $B
step vit_fwd 300 0 env FLUXMPI_GEMM_NT=fwd $B
step vit_lb0 300 0 env FLUXMPI_LINBWD=0 $B
step vit_b 300 0 $B
step vit_fwdb 300 0 env FLUXMPI_GEMM_NT=fwd $B
step vit_lb0b 300 0 env FLUXMPI_LINBWD=0 $B
for jr in 0.5,0.05 2.0,0.05; do
  step jr_deq_$jr 200 0 env FLUXMPI_DEQ_JR=$jr python scripts/diag_deq_contract.py --model deq --steps 40
  step jr_deqc_$jr 300 0 env FLUXMPI_DEQ_JR=$jr python scripts/diag_deq_contract.py --model deq_cifar --steps 40
done
echo done
