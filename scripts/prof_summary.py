#!/usr/bin/env python
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into markdown (top-N kernels, grouped categories).

usage: python scripts/prof_summary.py <kernel_stats.csv> [steps] [title] > profiles/<name>.md
"""
import csv
import re
import sys

CATS = [
    ("fluxmpi HIP (ours)", r"fluxmpi|mt_copy|mt_adam|mt_sgd|mt_fill|bn_stats|bn_norm|bn_bwd|adam_advance|mt_sumsq"),
    ("GEMM (hipBLASLt/Tensile)", r"^Cijk|^Custom_Cijk"),
    ("conv (MIOpen igemm/naive)", r"igemm|conv|Conv|naive"),
    ("MIOpen BatchNorm", r"MIOpenBatchNorm"),
    ("RCCL", r"ncclDevKernel|nccl|rccl"),
    ("attention", r"attn|flash|fmha"),
    ("torch elementwise/reduce", r"at::native"),
]


def cat_of(name):
    for c, rx in CATS:
        if re.search(rx, name):
            return c
    return "other"


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    title = sys.argv[3] if len(sys.argv) > 3 else path
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Total kernel time {tot / 1e6:.2f} ms over {steps:g} steps = **{tot / 1e6 / steps:.2f} ms/step**\n")
    cats = {}
    for r in rows:
        c = cat_of(r["Name"])
        cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
    print("| category | ms/step | % |\n|---|---|---|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {v / 1e6 / steps:.2f} | {100 * v / tot:.1f} |")
    print("\n| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        n = r["Name"]
        n = (n[:90] + "…") if len(n) > 90 else n
        print(f"| `{n}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
