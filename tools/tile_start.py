#!/usr/bin/env python3
"""Per-tile duration against start time within the frame (diagnostic;
RT_DIAG_TILECOST build via RT_LIB): is the start of the kernel (every wave at
the root at once) slower than its middle?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene
    tris, _ = sponza_scene()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    W, H = 1920, 1080
    tx, ty = (W + 7) // 8, (H + 7) // 8
    T = tx * ty
    path = rt.CameraPath(rt.scene_center(tris), 36)
    ids = torch.empty(W * H, dtype=torch.int32, device="cuda:0")
    hp = torch.zeros(12 * W * H, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    for F in (0, 12, 24):
        pos, d = path.circular_path(F)
        for rep in range(3):
            s.render_rows_device(0, pos, d, W, H, 0, 1, H, hit_id=ids.data_ptr(), hit_pos=hp.data_ptr(),
                                 stream=st.cuda_stream)
            torch.cuda.synchronize()
        a = hp[0:3 * T].cpu().numpy().reshape(-1, 3)
        sp = hp[3 * T:11 * T].cpu().numpy().reshape(-1, 8)
        dur = a[:, 0] / 100
        start = (sp[:, 6] - sp[:, 6].min()) / 100
        end = start + dur
        print(f"frame {F}: kernel span {end.max():.1f} us, tiles {T}")
        edges = np.arange(0, end.max() + 10, 10)
        for lo in edges[:-1]:
            m = (start >= lo) & (start < lo + 10)
            if m.sum() == 0:
                continue
            nodes = (a[m, 1] % 1e6).mean()
            print(f"  start {lo:5.0f}-{lo + 10:3.0f} us: tiles {m.sum():5d}  mean dur {dur[m].mean():6.1f}  "
                  f"max {dur[m].max():6.1f}  nodes {nodes:5.1f}  node-wait/node {sp[m, 0].mean() / max(nodes, 1):6.0f}")
        # active waves over time
        tt = np.arange(0, end.max(), 5)
        act = [(np.sum((start <= t) & (end > t))) for t in tt]
        print("  active tiles every 5 us:", " ".join(str(x) for x in act))


if __name__ == "__main__":
    main()
