#!/usr/bin/env python3
"""VALU issue utilisation of the traversal kernel from the rocprofv3 SQ passes
of `tools/gpu_session.sh sq` (north_star asks for VALU-utilisation counters
beside the HBM roofline).

  busy = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)

A wave64 VALU instruction occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md,
"Wave scheduling"); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  The non-
counting dispatch of one 36-frame launch is used.

Also the issue roofline of the kernel: the share of the
SIMDs' issue cycles its VALU and SALU instructions take,

  issue = (SQ_INSTS_VALU x 2 + SQ_INSTS_SALU x 1) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)

(a wave64 VALU instruction holds its SIMD-32 for 2 cycles, a SALU
instruction issues in 1), with the VALU and SALU shares beside it.

Usage: tools/pmc_valu.py [--kernel NAME] KEY_FILE OUT_JSON SQ_CSV [SQ_CSV ...]
  NAME: k_trace_packet (default), k_paths, or queue (the queued path tracer's
  kernels summed per pose)
"""
import collections
import csv
import os
import re
import json
import sys



def counting(name):
    """k_trace_packet<W, SP, K, COUNT, FUSED> / k_paths<W, S, COUNT, ...>: the
    COUNT instantiation is the counting pass, not the timed kernel."""
    m = re.search(r"k_trace_packet<\d+, \d+, \d+, (true|false)", name) or \
        re.search(r"k_paths<\d+, \d+, (true|false)", name)
    return bool(m and m.group(1) == "true")


def main():
    args = sys.argv[1:]
    kernel = "k_trace_packet"
    if args and args[0] == "--kernel":
        kernel = args[1]
        args = args[2:]
    key_file, out = args[:2]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    if kernel == "queue":  # the queued path tracer: its kernels summed per pose (pmc_traffic.per_pose)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pmc_traffic import per_pose
        for path in args[2:]:
            for pose, cs in per_pose(path).items():
                for c, v in cs.items():
                    tot[c] += v
                    disp[c].add((path, pose))
    for path in args[2:] if kernel != "queue" else []:
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if kernel + "<" not in n or counting(n):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((path, r["Dispatch_Id"]))
    per = {c: tot[c] / max(len(disp[c]), 1) for c in tot}  # per dispatch (queue: per pose)
    cycles = per["GRBM_GUI_ACTIVE"] / 8.0
    valu = per["SQ_INSTS_VALU"]
    salu = per.get("SQ_INSTS_SALU")
    res = {
        "workload_key": open(key_file).read().strip(),
        "kernel": kernel,
        "valu_insts_per_launch": valu,
        "salu_insts_per_launch": salu,
        "cycles_per_xcd": cycles,
        "valu_busy": round(valu * 2.0 / (1024.0 * cycles), 4),
        **({"issue": round((valu * 2.0 + salu) / (1024.0 * cycles), 4),
            "salu_share": round(salu / (1024.0 * cycles), 4)} if salu else {}),
        "wave_cycles_split": {k: round(per[k] / per["SQ_WAVE_CYCLES"], 4)
                              for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                        "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_ANY") if k in per},
        "method": "rocprofv3 --pmc SQ passes (tools/gpu_session.sh sq); busy = SQ_INSTS_VALU x 2 / "
                  "(1024 SIMDs x GRBM_GUI_ACTIVE/8)",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
