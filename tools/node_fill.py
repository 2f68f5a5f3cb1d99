#!/usr/bin/env python3
"""Wide-node fill of the traversal (diagnostic): fraction of wave node visits
to nodes with <= 4 valid child slots and mean valid slots per visit, from the
counting kernel's raw counters (rt_diag_raw words 7, 8, 13-15)."""
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
    W, H, F = 1920, 1080, 4
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f * 9) for f in range(F)]
    ids = torch.empty(F * W * H, dtype=torch.int32, device="cuda:0")
    s.frame_stats(0, reset=True)
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ids.data_ptr(), stream=torch.cuda.current_stream().cuda_stream,
                          count=True)
    torch.cuda.synchronize()
    raw = np.zeros(16, np.uint64)
    N.check(N.lib().rt_diag_raw(s.handle, 0, raw.ctypes.data, 16))
    nodes, empty_pop, popcull, empty = int(raw[7]), int(raw[13]), int(raw[14]), int(raw[15])
    print(f"wave node visits {nodes}: popped and empty {empty_pop / nodes:.3f}, pops culled {popcull}, "
          f"no child entered {empty / nodes:.3f}; leaf visits {int(raw[8])}")


if __name__ == "__main__":
    main()
