#!/usr/bin/env python3
"""FETCH_SIZE calibration for the headline kernel's read types.

Reads the rocprofv3 `--pmc FETCH_SIZE TCC_EA0_RDREQ_sum` pass over
tools/fetch_probe (2 GiB read once per probe kernel, the Infinity Cache
flushed in between) and writes, per probe, FETCH_SIZE in bytes (the counter is
in KiB), the read requests, and the factor that turns FETCH_SIZE into the
bytes actually read (known / FETCH_SIZE bytes).

Usage: tools/fetch_calib.py FETCH_CSV OUT_JSON [WRITE_CSV]
"""
import collections
import csv
import json
import sys

KNOWN = 2 << 30  # bytes each probe reads (tools/fetch_probe.hip)
PROBES = {"k_uniform32": "uniform (scalar) 32-B records, 8 per step: wide-node child records",
          "k_gather8": "8 B per lane, lanes permuted inside 512-B blocks",
          "k_rec72": "first 72 B of a 128-B record per lane (the resolve's fp64 Moller-Trumbore part)",
          "k_wide16": "16 B per lane, coalesced (MI355X_MICROARCH.md's calibrated case)"}
STORES = {"k_store4": ("4-B stores per lane, coalesced (hit ids)", KNOWN),
          "k_store8": ("8-B stores per lane, coalesced (fp64 distances)", KNOWN),
          "k_store3": ("3 one-byte stores per lane, coalesced (PPM colour bytes)", 3 * (KNOWN // 3))}


def main():
    path, out = sys.argv[1:3]
    wpath = sys.argv[3] if len(sys.argv) > 3 else None
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        for p in PROBES:
            if p in name:
                vals[p][r["Counter_Name"]] += float(r["Counter_Value"])
    res = {}
    for p, desc in PROBES.items():
        if p not in vals:
            continue
        fb = vals[p]["FETCH_SIZE"] * 1024.0
        rq = vals[p].get("TCC_EA0_RDREQ_sum", 0.0)
        res[p] = {"pattern": desc, "known_bytes": KNOWN, "fetch_size_bytes": round(fb),
                  "rdreq": round(rq), "bytes_per_rdreq": round(KNOWN / rq, 2) if rq else None,
                  "fetch_size_fraction_of_known": round(fb / KNOWN, 4),
                  "correction_factor": round(KNOWN / fb, 4) if fb else None}
    if wpath:
        wv = collections.defaultdict(float)
        for r in csv.DictReader(open(wpath)):
            for p in STORES:
                if p in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
                    wv[p] += float(r["Counter_Value"])
        for p, (desc, known) in STORES.items():
            if p in wv:
                wb = wv[p] * 1024.0
                res[p] = {"pattern": desc, "known_bytes": known, "write_size_bytes": round(wb),
                          "write_size_fraction_of_known": round(wb / known, 4),
                          "correction_factor": round(known / wb, 4) if wb else None}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum / --pmc WRITE_SIZE -- tools/fetch_probe",
               "probes": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
