#!/usr/bin/env python3
"""Are the expensive tiles slow on their own, or only next to the rest of the
frame?  (diagnostic; RT_DIAG_TILECOST build via RT_LIB)

Renders frame F of the bench orbit twice: the full 1920x1080 frame, and only
the band of image rows [R0, R0 + N) as its own launch.  Prints the per-tile
durations of the band's tiles in both runs and their cycle split.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene
    F = int(os.environ.get("F", "12"))
    R0, N = int(os.environ.get("R0", "152")), int(os.environ.get("N", "56"))
    tris, _ = sponza_scene()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    W, H = 1920, 1080
    tx = (W + 7) // 8
    path = rt.CameraPath(rt.scene_center(tris), 36)
    pos, d = path.circular_path(F)
    ids = torch.empty(W * H, dtype=torch.int32, device="cuda:0")
    hp = torch.zeros(12 * W * H, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()

    def run(row0, nrows):
        out = []
        for rep in range(3):
            hp.zero_()
            s.render_rows_device(0, pos, d, W, H, row0, 1, nrows, hit_id=ids.data_ptr(), hit_pos=hp.data_ptr(),
                                 stream=st.cuda_stream)
            torch.cuda.synchronize()
            tiles = tx * ((nrows + 7) // 8)
            a = hp[0:3 * tiles].cpu().numpy().reshape(-1, 3).copy()
            sp = hp[3 * tiles:11 * tiles].cpu().numpy().reshape(-1, 8)[:, :6].copy()
            out.append((a, sp))
        return out[-1]

    full, fsp = run(0, H)
    band, bsp = run(R0, N)
    t0 = (R0 // 8) * tx
    nt = (N // 8) * tx
    fb = full[t0:t0 + nt]
    fs = fsp[t0:t0 + nt]
    print(f"frame {F}: band rows [{R0},{R0 + N}) = {nt} tiles")
    for label, a, sp in (("in full frame", fb, fs), ("band alone", band[:nt], bsp[:nt])):
        c = a[:, 0] / 100
        top = np.argsort(-c)[:50]
        print(f"  {label:14s} mean {c.mean():7.1f} us  p90 {np.percentile(c, 90):7.1f}  max {c.max():7.1f}  "
              f"top50 {c[top].mean():7.1f}  | top50 split " + " ".join(f"{v:8.0f}" for v in sp[top].mean(axis=0)))
    print("  full-frame tile mean", full[:, 0].mean() / 100, "us, max", full[:, 0].max() / 100)


if __name__ == "__main__":
    main()
