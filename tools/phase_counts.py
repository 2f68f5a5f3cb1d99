#!/usr/bin/env python3
"""Dynamic per-phase instruction counts of the headline kernel (VERDICT r5
item 2: the static ISA counts treat rare paths as hot).

    python tools/phase_counts.py OUT.txt base=CSV split=CSV dblnode=CSV dblleaf=CSV [--stats JSON]

Each CSV is one rocprofv3 `--pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM
SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE` pass
over `bench.py --steps 1 --warmup 0 --frames 36` (one 36-pose launch per
timed dispatch) with one library:
  base     the shipped kernel (walk + fused resolve)
  split    RT_RESOLVE=split: the same walk handing its candidate lists to
           k_resolve (walk kernel and resolve kernel counted apart)
  dblnode  a measurement build that runs every node step's child test twice
           (RT_DBL_NODE: the second on an opaque copy of the culling distance,
           so the compiler cannot merge them; the traversal is unchanged)
  dblleaf  the same for the leaf's triangle filter (RT_DBL_LEAF)
The extra instructions of dblnode / dblleaf over base are the dynamic count
of that phase's test exactly (same tiles, same node steps and triangle
records); the walk-only kernel minus both is the rest of the walk (ray
set-up, stack pushes and pops, the leaf loop's control and candidate
appends); base minus the walk kernel is the fused resolve, shading and
stores (the split walk writes lists instead).  --stats: a bench JSON line
(per-tile node steps and triangle records) to express the tests per node
step and per triangle record.
"""
import collections
import csv
import json
import re
import sys

TILES = 36 * (1920 // 8) * (1080 // 8)  # tiles of one 36-pose 1080p launch
COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD")


def per_kernel(path):
    """{kernel name: {counter: mean per dispatch}} over the timed (non-counting) dispatches."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if re.search(r"k_trace_packet<\d+, \d+, \d+, true", n) or "k_resolve<true>" in n:
            continue  # the counting pass
        acc[n][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for n, d in acc.items():
        per = collections.defaultdict(float)
        disp = set()
        for (dis, c), v in d.items():
            per[c] += sum(v)
            disp.add(dis)
        out[n] = {c: per[c] / max(len(disp), 1) for c in per} | {"dispatches": len(disp)}
    return out


def pick(k, pat):
    c = [n for n in k if re.search(pat, n)]
    if not c:
        raise SystemExit(f"no kernel matching {pat}: {list(k)[:8]}")
    return k[max(c, key=lambda n: k[n]["dispatches"])]


def main():
    out = sys.argv[1]
    runs, stats = {}, None
    for a in sys.argv[2:]:
        if a.startswith("--stats="):
            l = [x for x in open(a.split("=", 1)[1]) if x.startswith("{")][-1]
            stats = json.loads(l)["roofline"]["per_ray"]
            continue
        k, v = a.split("=", 1)
        runs[k] = per_kernel(v)
    fused = r"k_trace_packet<8, 128, 8, false, true, false, false, false>"
    walk = r"k_trace_packet<8, 128, 8, false, false, false, false, false>"
    base = pick(runs["base"], fused)
    wk = pick(runs["split"], walk)
    rs = pick(runs["split"], r"k_resolve<false>")
    dn = pick(runs["dblnode"], fused)
    dl = pick(runs["dblleaf"], fused)
    rows = []
    for c in COUNTERS:
        t = lambda d: d.get(c, 0.0) / TILES
        node, leaf = t(dn) - t(base), t(dl) - t(base)
        rows.append((c, t(base), node, leaf, t(wk) - node - leaf, t(base) - t(wk), t(wk), t(rs)))
    lines = []
    w = lines.append
    w("# Dynamic instructions per 8x8 tile of k_trace_packet<8,128,8,false,true> (36-pose 1080p launch, "
      f"{TILES} tiles), from SQ counters of phase-doubled builds (tools/phase_counts.py)")
    w(f"{'counter':18s} {'total':>8s} {'node test':>10s} {'leaf filt':>10s} {'walk rest':>10s} "
      f"{'resolve+':>10s} | {'split walk':>10s} {'k_resolve':>10s}")
    for c, tot, node, leaf, rest, res, wkv, rsv in rows:
        w(f"{c:18s} {tot:8.1f} {node:10.1f} {leaf:10.1f} {rest:10.1f} {res:10.1f} | {wkv:10.1f} {rsv:10.1f}")
    w("")
    w("columns: total = the shipped kernel; node test = dblnode - base (the child slab tests, the any-mask fold);")
    w("leaf filt = dblleaf - base (tri_classify of every triangle record); walk rest = split walk kernel - node -")
    w("leaf (ray set-up, stack, near-child pick, leaf loop control, candidate appends, list hand-off);")
    w("resolve+ = base - split walk (fp64 resolve, chain check, shading, stores, hit counts, exit path)")
    if stats:
        ns, tr = stats["wave_nodes_per_tile"], stats["wave_tris_per_tile"]
        v = dict((r[0], r) for r in rows)
        w("")
        w(f"per node step ({ns} per tile): node test {v['SQ_INSTS_VALU'][2] / ns:.1f} VALU, "
          f"{v['SQ_INSTS_SALU'][2] / ns:.1f} SALU")
        w(f"per triangle record ({tr} per tile): filter {v['SQ_INSTS_VALU'][3] / tr:.1f} VALU, "
          f"{v['SQ_INSTS_SALU'][3] / tr:.1f} SALU")
        tv = v["SQ_INSTS_VALU"]
        w(f"VALU shares: node test {tv[2] / tv[1]:.1%}, leaf filter {tv[3] / tv[1]:.1%}, walk rest "
          f"{tv[4] / tv[1]:.1%}, resolve+ {tv[5] / tv[1]:.1%}")
        ts = v["SQ_INSTS_SALU"]
        w(f"SALU shares: node test {ts[2] / ts[1]:.1%}, leaf filter {ts[3] / ts[1]:.1%}, walk rest "
          f"{ts[4] / ts[1]:.1%}, resolve+ {ts[5] / ts[1]:.1%}")
    text = "\n".join(lines) + "\n"
    open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
