#!/usr/bin/env python3
"""HBM traffic per launch of the traversal kernel from rocprofv3 PMC passes.

Reads the FETCH_SIZE pass (with TCC_EA0_RDREQ_sum alongside, to pin the unit)
and the WRITE_SIZE pass written by `tools/gpu_session.sh pmc`, averages the
non-counting traversal-kernel dispatches and writes the JSON that bench.py
reads for `roofline.traffic`.

Correction: on gfx950 FETCH_SIZE reports half of the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section: 128-B requests tallied at
64 B).  tools/fetch_probe calibrates the other read types
(profiles/r03_fetch_calib.json): vector gathers (8 B per lane; the first 72 B
of 128-B records per lane) read 2 x FETCH_SIZE like the wide reads, but
uniform (scalar) loads are exact — 64-B requests, FETCH_SIZE x 1.  The packet
kernel reads its walk records (nodes, fp32 triangles) with scalar loads and
its fp64 resolve records with vector gathers, so with WALK_CSV (the same
launch with RT_RESOLVE=split, whose walk kernel reads by scalar loads only):
read bytes = F_walk + 2 (F_fused - F_walk); without it, 2 x FETCH_SIZE (an
upper bound for a kernel with scalar reads).  WRITE_SIZE is taken as is.

Usage: tools/pmc_traffic.py FETCH_CSV WRITE_CSV KEY_FILE OUT_JSON [KERNEL [WALK_CSV]]
(KERNEL: k_trace_packet, the default, k_paths for config c5's megakernel, or
"queue" for the queued path tracer: every k_q_* / k_sh_* dispatch of a pose
and its primary segments' packet kernel (k_trace_packet<..., PATHS = true>),
summed, per pose)
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


# the packet kernel's path-primary instantiation: k_trace_packet<W, SP, K,
# COUNT, FUSED, PACK, JOB, PATHS = true>
PACKET_PATHS = re.compile(r"k_trace_packet<\d+, \d+, \d+, (true|false), \w+, \w+, \w+, true>")
QUEUE = re.compile(r"k_q_|k_sh_|" + PACKET_PATHS.pattern)


def queue_counting(name):
    """The queued pipeline's COUNT instantiations (queue_paths.h):
    k_q_primary<W, S, COUNT, ..>, k_q_segment<W, S, K, COUNT, ..>,
    k_q_fallback<W, S, COUNT, ..>, k_sh_walk<W, COUNT>, k_sh_lane<W, S, COUNT>,
    and the packet kernel's path primaries."""
    m = (re.search(r"k_q_primary<\d+, \d+, (true|false)", name) or re.search(r"k_q_segment<\d+, \d+, \d+, (true|false)", name)
         or re.search(r"k_q_fallback<\d+, \d+, (true|false)", name) or re.search(r"k_sh_walk<\d+, (true|false)", name)
         or re.search(r"k_sh_lane<\d+, \d+, (true|false)", name) or PACKET_PATHS.search(name))
    return bool(m and m.group(1) == "true")


def pose_start(name):
    """A pose's first kernel: its primary segments (k_q_primary or the packet
    kernel's path primaries), not the counting instantiation."""
    return ("k_q_primary<" in name or bool(PACKET_PATHS.search(name))) and not queue_counting(name)


def per_pose(path):
    """KERNEL "queue": the queued path tracer's kernels summed per pose.  The
    counting pose (first) is skipped: every dispatch before the first
    non-counting primary-segment kernel; a pose starts at each (pose_start)."""
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        if not QUEUE.search(r["Kernel_Name"]):
            continue
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
    poses = collections.defaultdict(lambda: collections.defaultdict(float))
    pose = -1
    for d in sorted(rows):
        n = names[d]
        if pose_start(n):
            pose += 1
        if pose < 0 or queue_counting(n):
            continue
        for c, v in rows[d].items():
            poses[pose][c] += v
    return poses


def per_dispatch(path, kernel_sub):
    if kernel_sub == "queue":
        return per_pose(path)
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
    walk = None
    if len(sys.argv) > 6:
        wk = per_dispatch(sys.argv[6], kern)
        if wk:
            walk = sum(d["FETCH_SIZE"] for d in wk.values()) / len(wk)
    if walk is not None:
        # scalar walk reads at FETCH_SIZE x 1, the rest (vector) at x 2
        read_b = (walk + 2.0 * max(0.0, fetch - walk)) * unit
    else:
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
        **({"walk_only_fetch_size_avg": walk, "read_bytes_upper_bound": 2.0 * fetch * unit,
            "read_bytes_lower_bound": fetch * unit} if walk is not None else {}),
        "method": ("rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum / --pmc WRITE_SIZE, separate passes; " +
                   ("read = walk-only FETCH_SIZE x 1 (scalar loads, calibrated exact) + the fused kernel's "
                    "remaining FETCH_SIZE x 2 (vector gathers, calibrated x 2; profiles/r03_fetch_calib.json)"
                    if walk is not None else "read = 2 x FETCH_SIZE (gfx950 correction)") +
                   ", write = WRITE_SIZE"),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
