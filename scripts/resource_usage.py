#!/usr/bin/env python
"""Per-kernel register / scratch / LDS usage of one HIP source, compiled for gfx950 the way
``fluxmpi_amd/_build.py`` compiles it (``-Rpass-analysis=kernel-resource-usage``).

    python scripts/resource_usage.py csrc/kernels/gemm_nt.hip [--filter gemm_nt_kernel]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    from fluxmpi_amd import _build as B

    src = os.path.abspath(a.src)
    cmd = B._compile_cmd(src, "/tmp/_resource_usage.o") + ["-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr)
        return r.returncode
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for row in rows:
        if a.filter and a.filter not in row["name"]:
            continue
        print(f"{row.get('VGPRs', '?'):>4} vgpr {row.get('AGPRs', '?'):>3} agpr "
              f"{row.get('ScratchSize [bytes/lane]', '?'):>4} B scratch  occ {row.get('Occupancy [waves/SIMD]', '?')}  "
              f"lds {row.get('LDS Size [bytes/block]', '?'):>6}  {row['name'][:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
