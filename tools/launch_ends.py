#!/usr/bin/env python3
"""Where does each launch end?  (rocprofv3 kernel trace of bench.py)

    python tools/launch_ends.py TRACE_CSV [--out FILE]

For every timed traversal launch (k_trace_packet, not the counting
instantiation) lists the library kernels that follow it on the same queue
before that queue's next traversal launch (round 4: a k_fixup that could
only start once the other stream's persistent grid had drained), and how
long after the traversal kernel's end the launch's last library kernel
ended.  Round 5's packet kernel finishes the launch itself (packet_exit), so
the last kernel of a launch is its traversal kernel: 0 ms.
"""
import argparse
import csv
import re
import statistics

LIB = re.compile(r"\(anonymous namespace\)::k_")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    ap.add_argument("--timed", type=int, default=30, help="traversal launches of the timed region (bench.py --steps)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    t0 = ev[0][0]
    by_q = {}
    for e in ev:
        by_q.setdefault(e[3], []).append(e)
    lines = ["# launch start_ms trace_end_ms last_lib_kernel_end_ms tail_after_trace_ms queue followers",
             ]
    tails = []
    for q, es in by_q.items():
        idx = [k for k, e in enumerate(es) if "k_trace_packet<" in e[2] and ", false, true" in e[2]
               and not re.search(r"k_trace_packet<\d+, \d+, \d+, true", e[2])]
        for n, k in enumerate(idx):
            stop = idx[n + 1] if n + 1 < len(idx) else len(es)
            fol = [e for e in es[k + 1:stop] if LIB.search(e[2])]
            end = max([es[k][1]] + [e[1] for e in fol])
            tail = (end - es[k][1]) / 1e6
            tails.append(tail)
            names = ",".join(re.sub(r".*::(k_\w+).*", r"\1", e[2]) for e in fol) or "-"
            lines.append(f"{(es[k][0] - t0) / 1e6:10.3f} {(es[k][1] - t0) / 1e6:10.3f} {(end - t0) / 1e6:10.3f} "
                         f"{tail:8.4f} q{q} {names}")
    lines.append(f"# launches {len(tails)}; tail after the traversal kernel: max {max(tails):.4f} ms, "
                 f"median {statistics.median(tails):.4f} ms")
    # Launches on two streams overlap (launch k + 1's waves start on the CUs
    # launch k's tail frees), so a kernel's own start-to-end duration exceeds
    # the time per launch; the union of the last `timed` traversal launches'
    # busy intervals, per launch, is the figure bench.py's roofline divides by.
    trav = sorted((e[0], e[1]) for e in ev if "k_trace_packet<" in e[2] and ", false, true" in e[2]
                  and not re.search(r"k_trace_packet<\d+, \d+, \d+, true", e[2]))[-a.timed:]
    if trav:
        busy, (cs, ce) = 0, trav[0]
        for s0, e0 in trav[1:]:
            if s0 > ce:
                busy, cs, ce = busy + ce - cs, s0, e0
            else:
                ce = max(ce, e0)
        busy += ce - cs
        durs = sorted((e0 - s0) / 1e6 for s0, e0 in trav)
        lines.append(f"# last {len(trav)} traversal launches: busy union {busy / 1e6 / len(trav):.4f} ms per launch, "
                     f"own duration median {statistics.median(durs):.4f} ms (overlapped)")
    text = "\n".join(lines) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    print(text[-400:])


if __name__ == "__main__":
    main()
