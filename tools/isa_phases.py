#!/usr/bin/env python3
"""Instruction accounting of the headline kernel at the ISA level.

    python tools/isa_phases.py [lib.so] [--kernel MANGLED_SUBSTR] [--out FILE]

Disassembles the gfx950 code object of the built library and splits the
timed instantiation k_trace_packet<8,128,8,false,true,false,false> into the
phases its wave priorities mark (packet_kernel.h: `s_setprio 0` node steps,
`s_setprio 1` leaf visits, `s_setprio 2` the epilogue — resolve, stores,
the next tile's claim and ray set-up).  For the first octant copy of the
walk it prints the node step (from its four `s_load_dwordx16` to the branch
back) and one leaf chunk (two triangle records) instruction by instruction,
each with its class, then per-class counts per phase.  Classes: VALU, SALU,
SMEM (scalar loads), VMEM (global/buffer/scratch), LDS, BR (branches),
WAIT (s_waitcnt), NOP (s_nop: hazard padding), SPILL (v_readlane /
v_writelane of the SGPR spill VGPRs).
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import LLVM, code_objects  # noqa: E402

HEADLINE = "k_trace_packetILi8ELi128ELi8ELb0ELb1ELb0ELb0E"


def classify(mn: str, ops: str) -> str:
    if mn.startswith("s_waitcnt"):
        return "WAIT"
    if mn == "s_nop":
        return "NOP"
    if mn.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
        return "BR"
    if mn.startswith(("s_load", "s_buffer_load", "s_store", "s_memtime", "s_dcache")):
        return "SMEM"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if mn.startswith("ds_"):
        return "LDS"
    if mn in ("v_readlane_b32", "v_writelane_b32"):
        # SGPR spill slots live in lanes of dedicated VGPRs (v70/v71 in the
        # round-5 build); lane moves of the walk's own refs are VALU work
        m = re.match(r"(v\d+|s\d+)", ops.strip())
        return "SPILL" if m and m.group(1) in SPILL_VGPRS else "VALU"
    if mn.startswith("v_"):
        return "VALU"
    if mn.startswith("s_"):
        return "SALU"
    return "OTHER"


SPILL_VGPRS = set()


def disasm(lib: str, key: str):
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], capture_output=True,
                                 text=True).stdout
            lines = out.splitlines()
            for i, ln in enumerate(lines):
                if ln.endswith(">:") and key in ln and not re.search(r"<L\d+>:$", ln):
                    j = i + 1
                    while j < len(lines) and not (lines[j].endswith(">:") and not re.search(r"<L\d+>:$", lines[j])):
                        j += 1
                    return lines[i:j]
    raise SystemExit(f"kernel {key} not found in {lib}")


def instrs(lines):
    """(index, mnemonic, operands, text) of every instruction line."""
    out = []
    for i, ln in enumerate(lines):
        m = re.match(r"\t([a-z_0-9]+)\s*(.*?)\s*//", ln)
        if m:
            out.append((i, m.group(1), m.group(2), ln.split("//")[0].rstrip()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                           "raytracingdemo_amd", "librtmi355x.so"))
    ap.add_argument("--kernel", default=HEADLINE)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = disasm(a.lib, a.kernel)
    ins = instrs(lines)
    # spill VGPRs: targets of v_writelane_b32 with a constant lane >= 8
    for _, mn, ops, _ in ins:
        if mn == "v_writelane_b32":
            m = re.match(r"(v\d+),\s*s\d+,\s*(\d+)$", ops)
            if m and int(m.group(2)) >= 8:
                SPILL_VGPRS.add(m.group(1))
    for _, mn, ops, _ in ins:
        if mn == "v_readlane_b32":
            m = re.match(r"s\d+,\s*(v\d+),\s*(\d+)$", ops)
            if m and int(m.group(2)) >= 8:
                SPILL_VGPRS.add(m.group(1))
    # phases by the wave priority in force (straight-line order of the code)
    prio = 2
    phase_of = []
    for _, mn, ops, _ in ins:
        if mn == "s_setprio":
            prio = int(ops)
        phase_of.append(prio)
    names = {0: "node steps (prio 0)", 1: "leaf visits (prio 1)", 2: "set-up, resolve, stores (prio 2)"}
    tot = collections.defaultdict(collections.Counter)
    for (_, mn, ops, _), ph in zip(ins, phase_of):
        tot[ph][classify(mn, ops)] += 1
    out = []
    w = out.append
    w(f"# ISA accounting of {a.kernel} ({os.path.basename(a.lib)})")
    w(f"# spill VGPRs (SGPR spill lanes): {sorted(SPILL_VGPRS)}")
    w("")
    w("## Static instruction counts per phase (all 9 octant copies of the walk)")
    cls = ["VALU", "SALU", "SMEM", "VMEM", "LDS", "BR", "WAIT", "NOP", "SPILL", "OTHER"]
    w(f"{'phase':36s} " + " ".join(f"{c:>6s}" for c in cls))
    for ph in (0, 1, 2):
        w(f"{names[ph]:36s} " + " ".join(f"{tot[ph][c]:6d}" for c in cls))
    # the first octant copy: node step = from the 4 s_load_dwordx16 of a node
    # to the branch that closes the step; leaf chunk = the s_load_dwordx16 +
    # s_load_dwordx8 of two triangle records to the loop's back edge
    first_node = next(k for k, (_, mn, ops, _) in enumerate(ins) if mn == "s_load_dwordx16" and phase_of[k] == 0)
    k = first_node
    while not (ins[k][1] == "s_branch" and phase_of[k] == 0 and k > first_node + 60):
        k += 1
    node_end = k
    # back up to the loop head label (the compare before the loads)
    node_start = first_node
    while node_start > 0 and ins[node_start - 1][1] in ("s_lshl_b32", "s_cbranch_scc1", "s_cmp_lt_i32"):
        node_start -= 1
    first_leaf = next(k for k in range(node_end, len(ins)) if ins[k][1].startswith("s_load_dword") and phase_of[k] == 1)
    # the leaf loop of copy 0 runs to the next priority change (the return
    # to the node steps)
    leaf_end = next(k for k in range(first_leaf, len(ins)) if ins[k][1] == "s_setprio") - 1

    def listing(a0, a1, title):
        c = collections.Counter()
        w("")
        w(f"## {title}")
        for kk in range(a0, a1 + 1):
            _, mn, ops, text = ins[kk]
            cl = classify(mn, ops)
            c[cl] += 1
            w(f"  {cl:5s} {text.strip()}")
        w("  counts: " + ", ".join(f"{x} {c[x]}" for x in cls if c[x]))
        return c

    cn = listing(node_start, node_end, "Node step, octant copy 0 (loop head to the branch back; both the pushing "
                                       "and the non-pushing path are listed)")
    cl = listing(first_leaf, leaf_end, "Leaf loop, octant copy 0: the body for one chunk of two triangle records "
                                       "(tri_classify per record, LDS candidate append, pool chunk path) and the "
                                       "loop control")
    text = "\n".join(out) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    print(text if not a.out else f"wrote {a.out}: node step {dict(cn)}, leaf chunk {dict(cl)}")


if __name__ == "__main__":
    main()
