#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches).

Usage: tools/pmc_summary.py CSV [CSV ...] [--match SUBSTR] [--per N]
  --match  only kernels whose name contains SUBSTR (default: k_trace)
  --per    also divide every counter by N (e.g. tiles traced) for per-unit rates
"""
import argparse
import collections
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="k_trace")
    ap.add_argument("--per", type=float, default=0.0)
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in a.csv:
        for row in csv.DictReader(open(path)):
            name = row["Kernel_Name"]
            if a.match not in name:
                continue
            short = name.replace("void (anonymous namespace)::", "").split("(")[0]
            tot[short][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[short].add((path, row["Dispatch_Id"]))
    for k, cs in tot.items():
        print(f"{k}  dispatches={len(disp[k])}")
        for c in sorted(cs):
            v = cs[c]
            extra = f"   per-unit {v / a.per:.1f}" if a.per else ""
            print(f"  {c:32s} {v:18.0f}{extra}")
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS"):
                if c in cs:
                    print(f"  {c:32s} {100 * cs[c] / wc:6.1f} % of wave cycles")


if __name__ == "__main__":
    main()
