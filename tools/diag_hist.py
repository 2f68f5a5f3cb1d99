#!/usr/bin/env python3
"""Per-tile cost histograms from an RT_DIAG_HIST build (diagnostic only).

Renders a few frames of the bench workload through the library named by
RT_LIB and prints the tile-duration histogram (2-us bins) and the summed
tile time per horizontal and vertical band of the image.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import raytracingdemo_amd as rt
    from raytracingdemo_amd import _native as N
    from raytracingdemo_amd.scenes import sponza_scene
    tris, _ = sponza_scene()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    W, H = 1920, 1080
    path = rt.CameraPath(rt.scene_center(tris), 36)
    ids = torch.empty(W * H, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream()
    frames = [0, 9, 18, 27]
    for f in frames:  # warm-up
        pos, d = path.circular_path(f)
        s.render_rows_device(0, pos, d, W, H, 0, 1, H, hit_id=ids.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    L = N.lib()
    # read the raw diagnostic block through rt_frame_stats' reset cycle is not
    # enough (it only returns sums), so use a dedicated copy of d_counters:
    # the histogram lives in the spread slots, returned via a second struct read
    s.frame_stats(0, reset=True)
    for f in frames:
        pos, d = path.circular_path(f)
        s.render_rows_device(0, pos, d, W, H, 0, 1, H, hit_id=ids.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    raw = (C.c_uint64 * (16 + 16 + 64 * 8))()
    N.check(L.rt_diag_raw(s.handle, 0, raw, len(raw)))
    slots = np.array(raw[32:]).reshape(64, 8)
    hist = slots[:, 4]
    print("tile duration histogram (2-us bins, count over", len(frames), "frames):")
    for b in range(64):
        if hist[b]:
            print(f"  {2*b:4d}-{2*b+2:4d} us: {int(hist[b]):6d}")
    tot = slots[:, 5].astype(float)
    print("summed tile time by image-row band (top -> bottom, % of total):")
    print("  " + " ".join(f"{100*x/tot.sum():.1f}" for x in tot))
    col = slots[:, 6].astype(float)
    print("by column band (left -> right):")
    print("  " + " ".join(f"{100*x/col.sum():.1f}" for x in col))


if __name__ == "__main__":
    main()
