#!/usr/bin/env python3
"""HBM traffic per launch of the traversal kernel from rocprofv3 PMC passes.

Reads the FETCH_SIZE pass (with TCC_EA0_RDREQ_sum alongside, to pin the unit)
and the WRITE_SIZE pass written by `tools/gpu_session.sh pmc`, averages the
non-counting traversal-kernel dispatches and writes the JSON that bench.py
reads for `roofline.traffic`.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half of the bytes of wide coalesced reads (128-B requests tallied at 64 B), so
read bytes = 2 x FETCH_SIZE; WRITE_SIZE is taken as is.

Usage: tools/pmc_traffic.py FETCH_CSV WRITE_CSV KEY_FILE OUT_JSON [KERNEL]
(KERNEL: k_trace_packet, the default, or k_paths for config c5)
"""
import collections
import csv
import re
import json
import sys



def counting(name):
    """k_trace_packet<W, SP, K, COUNT, FUSED> / k_paths<W, S, COUNT>: the COUNT
    instantiation is the counting pass, not the timed kernel."""
    m = re.search(r"k_trace_packet<\d+, \d+, \d+, (true|false)", name) or re.search(r"k_paths<\d+, \d+, (true|false)", name)
    return bool(m and m.group(1) == "true")


def per_dispatch(path, kernel_sub):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if kernel_sub not in name or counting(name):  # skip the counting variant
            continue
        vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return vals


def main():
    fetch_csv, write_csv, key_file, out = sys.argv[1:5]
    key = open(key_file).read().strip()
    kern = sys.argv[5] if len(sys.argv) > 5 else "k_trace_packet"
    f = per_dispatch(fetch_csv, kern)
    w = per_dispatch(write_csv, kern)
    if not f or not w:
        raise SystemExit("no traversal-kernel dispatches in the PMC CSVs")
    fetch = sum(d["FETCH_SIZE"] for d in f.values()) / len(f)
    rdreq = sum(d.get("TCC_EA0_RDREQ_sum", 0.0) for d in f.values()) / len(f)
    write = sum(d["WRITE_SIZE"] for d in w.values()) / len(w)
    # unit: rocprofv3 derives FETCH_SIZE / WRITE_SIZE in KiB; confirm against
    # the raw request count (FETCH_SIZE = RDREQ x 64 B per the guide)
    unit = 1024.0
    if rdreq > 0:
        ratio = fetch / (rdreq * 64.0)
        unit = 1.0 if abs(ratio - 1.0) < 0.25 else 1024.0
    read_b = 2.0 * fetch * unit
    write_b = write * unit
    res = {
        "workload_key": key,
        "kernel": kern,
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
        "fetch_size_avg": fetch, "write_size_avg": write, "tcc_ea0_rdreq_avg": rdreq,
        "unit_bytes": unit,
        "read_bytes_per_launch": read_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "method": "rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum / --pmc WRITE_SIZE, separate passes; "
                  "read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
