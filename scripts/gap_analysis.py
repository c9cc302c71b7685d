#!/usr/bin/env python
"""Idle gaps of the GPU over the last N steps of a rocprofv3 kernel trace.

Lists the largest gaps between consecutive kernels (on any queue) with the kernels on both sides,
and totals per-kernel-name time for names matching a pattern (e.g. ``mt_copy|nccl``).

usage: python scripts/gap_analysis.py <kernel_trace.csv> [N] [pattern]
"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_advance" in r["Kernel_Name"]]
    lo, hi = ends[-nsteps - 1] + 1, ends[-1] + 1
    win = rows[lo:hi]
    gaps = []
    busy_end = int(win[0]["End_Timestamp"])
    prev = win[0]
    for r in win[1:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > busy_end:
            gaps.append((s - busy_end, prev["Kernel_Name"][:70], r["Kernel_Name"][:70]))
        if e > busy_end:
            busy_end, prev = e, r
    tot = sum(g[0] for g in gaps)
    wall = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
    print(f"wall {wall / 1e6 / nsteps:.3f} ms/step, idle {tot / 1e6 / nsteps:.3f} ms/step in {len(gaps) / nsteps:.0f} gaps/step")
    gaps.sort(reverse=True)
    for g, a, b in gaps[:25]:
        print(f"{g / 1e3:8.1f} us  after {a}\n{'':13}before {b}")
    if pat:
        agg: dict = {}
        for r in win:
            if pat.search(r["Kernel_Name"]):
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                k = r["Kernel_Name"][:80]
                c, t = agg.get(k, (0, 0))
                agg[k] = (c + 1, t + d)
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{c / nsteps:6.1f}/step {t / 1e3 / nsteps:8.1f} us/step  {k}")


if __name__ == "__main__":
    main()
