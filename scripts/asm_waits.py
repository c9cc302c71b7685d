"""Count memory waits / loads after the last MFMA (the epilogue) of each kernel in a device .s file.

A load under a branch (``x = cond ? load(p) : 0``) makes the waitcnt pass wait for it at the join:
many ``vmcnt(0)`` here next to as many loads is the signature of serialized epilogue latency.

usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc --cuda-device-only -S -o /tmp/k.s csrc/kernels/gemm_glds.hip
       python scripts/asm_waits.py /tmp/k.s [kernel-name substring]
"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "gemm_glds_kernel"
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
for i, (st, name) in enumerate(starts):
    if pat not in name:
        continue
    body = s[st:starts[i + 1][0] if i + 1 < len(starts) else len(s)]
    body = body[:body.find("s_endpgm")]
    idx = body.rfind("v_mfma")
    epi = body[idx:]
    n0 = len(re.findall(r"vmcnt\(0\)", epi))
    nw = len(re.findall(r"s_waitcnt[^\n]*vmcnt", epi))
    nl = len(re.findall(r"global_load_dwordx4", epi))
    nb = len(re.findall(r"global_load_ubyte", epi))
    br = len(re.findall(r"s_cbranch", epi))
    short = re.search(r"kernelI(.*)EEvNS0", name)
    print(f"{short.group(1) if short else name[:60]:40s} epi: vmcnt0={n0:3d} vmwaits={nw:3d} ld16={nl:3d} ldb={nb:3d} br={br:3d}")
