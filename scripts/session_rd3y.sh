#!/bin/bash
# rd3y: which hipBLASLt epilogues have gfx950 solutions (ROCm 7.2's library and torch's bundled one)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
TL=$(python -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
mkdir -p /tmp/tl && ln -sf "$TL/libhipblaslt.so" /tmp/tl/libhipblaslt.so.1
step probe_rocm 120 0 ./scripts/probe/blaslt_probe_rocm
step probe_torch 120 0 env LD_LIBRARY_PATH=/tmp/tl HIPBLASLT_TENSILE_LIBPATH="$TL/hipblaslt/library" ./scripts/probe/blaslt_probe_torch
echo done
