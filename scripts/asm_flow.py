#!/usr/bin/env python
"""Print the memory / wait / branch skeleton of one kernel in a device .s file (runs of MFMAs,
LDS ops and DMA collapsed): a quick look at where a kernel waits for which loads.

usage: python scripts/asm_flow.py <file.s> <kernel-name substring> [max lines]
"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 200
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
KEYS = ("global_load", "global_store", "global_atomic", "s_waitcnt", "s_barrier", "s_cbranch", "s_branch",
        "buffer_", "v_mfma", "ds_", ".LBB")
for i, (st, name) in enumerate(starts):
    if pat not in name:
        continue
    body = s[st:starts[i + 1][0] if i + 1 < len(starts) else len(s)]
    body = body[:body.find("s_endpgm")]
    out, prev, cnt = [], None, 0
    for line in body.split("\n"):
        t = line.strip().split(";")[0].strip()
        if not t or not any(k in t for k in KEYS):
            continue
        op = t.split()[0]
        if op == prev and (op.startswith("v_mfma") or op.startswith("ds_") or "lds" in t):
            cnt += 1
            continue
        if cnt > 1:
            out.append(f"    x{cnt}")
        out.append(t[:90])
        prev, cnt = op, 1
    print(name)
    print("\n".join(out[:limit]))
    break
