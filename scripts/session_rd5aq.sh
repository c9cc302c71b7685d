#!/bin/bash
# round 5: gemm_nt built WITH SLP vectorisation (the round-4 NaN in EPI 1's gelu'(h) output, ADVICE
# round 4 medium): the EPI 1 diagnostic at the ViT shapes for both GELU forms, and the gemm_nt /
# GELU / ViT GPU tests, each against the default build and the SLP build
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
V=exp/variants/_C_gnt_slp.so
step epi1_noslp 180 0 python scripts/diag_epi1.py
step epi1_slp 180 0 env FLUXMPI_C_VARIANT=$V python scripts/diag_epi1.py
P="python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_gelu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread"
step tests_slp 600 0 env FLUXMPI_C_VARIANT=$V $P
echo done
