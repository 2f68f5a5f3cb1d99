#!/usr/bin/env python3
"""Per-tile traversal durations of the bench orbit (RT_DIAG_TILECOST build)
and simulated makespans of tile orders (diagnostic only).

Greedy list scheduling of the measured tile durations on P persistent waves,
in: row-major order (as shipped), true longest-first (oracle), the previous
frame's cost at the same tile, and the previous frame's cost shifted by the
orbit's image motion.  Writes gpurun_out/tile_costs.npz.
"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def makespan(costs, order, P):
    h = [0.0] * P
    heapq.heapify(h)
    for t in order:
        f = heapq.heappop(h)
        heapq.heappush(h, f + costs[t])
    return max(h)


def main():
    import torch
    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene
    tris, _ = sponza_scene()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    W, H = 1920, 1080
    tx, ty = (W + 7) // 8, (H + 7) // 8
    path = rt.CameraPath(rt.scene_center(tris), 36)
    ids = torch.empty(W * H, dtype=torch.int32, device="cuda:0")
    hp = torch.zeros(3 * W * H, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    costs, split = [], []
    for rep in range(2):
        for f in range(36):
            pos, d = path.circular_path(f)
            s.render_rows_device(0, pos, d, W, H, 0, 1, H, hit_id=ids.data_ptr(), hit_pos=hp.data_ptr(),
                                 stream=st.cuda_stream)
            torch.cuda.synchronize()
            if rep == 1:
                costs.append(hp[0:3 * tx * ty].cpu().numpy().reshape(-1, 3).copy())
                split.append(hp[3 * tx * ty:11 * tx * ty].cpu().numpy().reshape(-1, 8)[:, :6].copy())
    A = np.stack(costs)  # [36, tiles, 3]: 10-ns ticks, nodes + 1e6 leaves, triangles
    S = np.stack(split)  # [36, tiles, 6]: s_memtime split (node wait, node work, leaves, pops, setup, out)
    names = ["node-wait", "node-work", "leaves", "pops", "setup", "out"]
    for f in (0, 12, 30):
        top = np.argsort(-A[f, :, 0])[:100]
        for label, sel in (("all", slice(None)), ("top100", top)):
            sp = S[f][sel].mean(axis=0)
            nodes = (A[f][sel, 1] % 1e6).mean()
            leaves = (A[f][sel, 1] // 1e6).mean()
            tris = A[f][sel, 2].mean()
            print(f"f{f:2d} {label:7s} us {A[f][sel, 0].mean() / 100:6.1f} nodes {nodes:5.1f} leaves {leaves:5.1f} "
                  f"tris {tris:5.1f} | " + " ".join(f"{n} {v:8.0f}" for n, v in zip(names, sp)) +
                  f" | per-node wait {sp[0] / max(nodes, 1):6.0f} per-tri {sp[2] / max(tris, 1):6.0f}")
    C = A[:, :, 0]
    np.savez_compressed("gpurun_out/tile_costs.npz", costs=C, visits=A[:, :, 1], tris=A[:, :, 2], split=S, tx=tx, ty=ty)
    P = 7168
    print("tiles", tx * ty, "mean tile us", C.mean() / 100, "p99", np.percentile(C, 99) / 100)
    print("frame sum/P (ideal) vs row-major vs LPT-oracle vs prev-frame vs prev-frame shifted (us):")
    for f in range(0, 36, 6):
        c = C[f]
        ideal = c.sum() / P
        rm = makespan(c, range(len(c)), P)
        lpt = makespan(c, np.argsort(-c), P)
        prev = C[f - 1]
        pf = makespan(c, np.argsort(-prev), P)
        best_sh, best = 0, None
        for sh in range(-40, 41, 2):
            p2 = np.roll(prev.reshape(ty, tx), sh, axis=1).reshape(-1)
            m = makespan(c, np.argsort(-p2), P)
            if best is None or m < best:
                best, best_sh = m, sh
        corr = np.corrcoef(c, prev)[0, 1]
        print(f"  f{f:2d}: ideal {ideal/100:6.1f} rowmajor {rm/100:6.1f} lpt {lpt/100:6.1f} "
              f"prev {pf/100:6.1f} prev-shift({best_sh:+d}) {best/100:6.1f}  corr {corr:.2f}")


if __name__ == "__main__":
    main()
