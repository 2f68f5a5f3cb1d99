#!/usr/bin/env python3
"""Per-kernel attribution of one rocprofv3 PMC counter over a bench run.

    python tools/pmc_kernels.py COUNTER_CSV [--counter WRITE_SIZE] [--scale 1024]
                                [--per N] [--match REGEX] [--payload NAME=BYTES ...]

Sums the counter per kernel name (template arguments kept, so the counting
instantiations stay apart from the timed ones), divides by --per (e.g. the
poses or launches the run traced) and prints dispatches, total and per
dispatch.  WRITE_SIZE / FETCH_SIZE are in KiB units on gfx950 (--scale 1024
gives bytes; FETCH_SIZE also needs the x2 read correction of
tools/pmc_traffic.py, which this tool does not apply).  --payload gives a
kernel's legitimate bytes per dispatch (a substring of its name = bytes) to
print the excess beside it.
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--counter", default="WRITE_SIZE")
    ap.add_argument("--scale", type=float, default=1024.0)
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--match", default="")
    ap.add_argument("--payload", nargs="*", default=[])
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(a.csv)):
        if r["Counter_Name"] != a.counter or not re.search(a.match, r["Kernel_Name"]):
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        k = re.sub(r"\(.*\)$", "", k)
        tot[k] += float(r["Counter_Value"]) * a.scale
        n[k] += 1
    pay = dict(p.split("=", 1) for p in a.payload)
    print(f"{'kernel':60s} {'disp':>5s} {'GB/' + ('unit' if a.per != 1 else 'run'):>10s} {'GB/disp':>9s}")
    for k in sorted(tot, key=lambda k: -tot[k]):
        line = f"{k[:60]:60s} {n[k]:5d} {tot[k] / a.per / 1e9:10.3f} {tot[k] / n[k] / 1e9:9.3f}"
        for s, b in pay.items():
            if s in k:
                line += f"   payload {float(b) / 1e9:.3f} GB/disp, excess {tot[k] / n[k] / float(b):.2f}x"
        print(line)


if __name__ == "__main__":
    main()
