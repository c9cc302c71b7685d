#!/usr/bin/env python
"""Per-kernel stats over the LAST N training steps of a rocprofv3 kernel trace.

Warm-up (MIOpen find, first-call compiles) pollutes ``kernel_stats.csv``; the
steady state is the tail. Steps are delimited by the fused-Adam kernel
(``mt_adam_kernel``, launched once per bucket at the end of every step).

usage: python scripts/trace_window.py <kernel_trace.csv> [N] [title] > profiles/<name>.md
"""
import csv
import re
import sys

from prof_summary import cat_of


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    title = sys.argv[3] if len(sys.argv) > 3 else path
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # step boundary = last optimiser kernel of a step (the advance kernel), else last mt_adam
    ends = [i for i, r in enumerate(rows) if "adam_advance" in r["Kernel_Name"]]
    if len(ends) < nsteps + 1:
        ends = [i for i, r in enumerate(rows) if "mt_adam" in r["Kernel_Name"]]
    lo, hi = ends[-nsteps - 1] + 1, ends[-1] + 1
    win = rows[lo:hi]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    stats: dict = {}
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n = re.sub(r"\s+", " ", r["Kernel_Name"])
        s = stats.setdefault(n, [0, 0])
        s[0] += 1
        s[1] += d
    busy = sum(v[1] for v in stats.values())
    print(f"# {title}\n")
    print(f"Last {nsteps} steps: wall {1e-6 * (t1 - t0) / nsteps:.2f} ms/step, kernel busy "
          f"{1e-6 * busy / nsteps:.2f} ms/step ({len(win) // nsteps} kernels/step)\n")
    cats: dict = {}
    for n, (c, d) in stats.items():
        cats[cat_of(n)] = cats.get(cat_of(n), 0) + d
    print("| category | ms/step | % of busy |\n|---|---|---|")
    for c, d in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {1e-6 * d / nsteps:.2f} | {100 * d / busy:.1f} |")
    print("\n| kernel | calls/step | ms/step | avg us |\n|---|---|---|---|")
    for n, (c, d) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:40]:
        short = (n[:100] + "…") if len(n) > 100 else n
        print(f"| `{short}` | {c / nsteps:g} | {1e-6 * d / nsteps:.3f} | {1e-3 * d / c:.1f} |")


if __name__ == "__main__":
    main()
