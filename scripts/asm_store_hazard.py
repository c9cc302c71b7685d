#!/usr/bin/env python
"""Scan the gfx950 ISA of a HIP source for 16-B vector stores whose data VGPRs a later VALU (or
VMEM/LDS load) rewrites within N instructions — the epilogue store-data hazard of
profiles/rd5c_gemm_nt_store_hazard.md.  python scripts/asm_store_hazard.py csrc/kernels/*.hip [--window 3]"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STORE = re.compile(r"\s*(buffer|global)_store_dwordx4 v\[(\d+):(\d+)\]")
DST = re.compile(r"\s*(v_\S+|ds_read\S*|buffer_load\S*|global_load\S*)\s+(v\[(\d+):(\d+)\]|v(\d+))")


def scan(asm: str, window: int):
    lines = asm.split("\n")
    out = {}
    fn = None
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            fn = m.group(1)
        m = STORE.match(l)
        if not m or fn is None:
            continue
        data = set(range(int(m.group(2)), int(m.group(3)) + 1))
        n, j = 0, i + 1
        while n < window and j < len(lines):
            t = lines[j].strip()
            j += 1
            if not t or t.startswith((";", ".")):
                continue
            if t.startswith("s_nop"):
                n += int(t.split()[1]) + 1
                continue
            n += 1
            d = DST.match(t)
            if d and not d.group(1).startswith(("v_readfirstlane", "v_cmp")):
                regs = set(range(int(d.group(3)), int(d.group(4)) + 1)) if d.group(3) else {int(d.group(5))}
                if regs & data:
                    out[fn] = out.get(fn, 0) + 1
                    break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("srcs", nargs="+")
    ap.add_argument("--window", type=int, default=3)
    a = ap.parse_args()
    from fluxmpi_amd import _build as B
    for src in a.srcs:
        with tempfile.TemporaryDirectory() as td:
            s_out = os.path.join(td, "k.s")
            cmd = [c for c in B._compile_cmd(os.path.abspath(src), s_out) if c != "-c"] + ["-S", "--cuda-device-only"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                print(src, "compile failed", r.stderr[-400:])
                continue
            res = scan(open(s_out).read(), a.window)
        tot = sum(res.values())
        print(f"{os.path.basename(src)}: {tot} stores with data rewritten within {a.window} states "
              f"in {len(res)} kernels")
        for fn, n in sorted(res.items(), key=lambda kv: -kv[1])[:6]:
            print(f"    {n:4d}  {fn[:100]}")


if __name__ == "__main__":
    main()
