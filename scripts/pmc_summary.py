#!/usr/bin/env python
"""Per-kernel averages of a rocprofv3 --pmc run (``*_counter_collection.csv``: one row per
counter per dispatch) as a markdown table, with the derived wave-state shares
(WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY of WAVE_CYCLES; MFMA-busy share of BUSY cycles) when
those counters are present.

usage: python scripts/pmc_summary.py <counter_collection.csv> [kernel-name regex] > profiles/<name>.md
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "?")
        if pat is not None and not pat.search(name):
            continue
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in per.items():
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[-80:]
        print(f"### `{short}`\n")
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print("| counter | mean per dispatch | dispatches |\n|---|---|---|")
        for c in sorted(avg):
            print(f"| {c} | {avg[c]:.4g} | {len(cs[c])} |")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    print(f"| {c} / SQ_WAVE_CYCLES | {avg[c] / wc:.3f} | |")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
            print(f"| SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES | {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / avg['SQ_BUSY_CYCLES']:.3f} | |")
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            print(f"| SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE | {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f} | |")
        print()


if __name__ == "__main__":
    main()
