#!/usr/bin/env python3
"""Wave start / end spread of the persistent traversal kernel (diagnostic;
RT_DIAG_WAVES build selected with RT_LIB).  Renders one 12-frame batch of the
bench workload and prints, per launch, the spread of wave start and end times
relative to the earliest start, and tiles per wave."""
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
    W, H, F = 1920, 1080, 12
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(F)]
    ids = torch.empty(F * W * H, dtype=torch.int32, device="cuda:0")
    hp = torch.zeros(3 * 65536, dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    for rep in range(3):
        hp.zero_()
        s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ids.data_ptr(), hit_pos=hp.data_ptr(),
                              stream=st.cuda_stream)
        torch.cuda.synchronize()
    a = hp.cpu().numpy().reshape(-1, 3)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    start = (a[:, 0] - t0) / 100.0  # us
    end = (a[:, 1] - t0) / 100.0
    T = end.max()
    q = [0, 1, 10, 50, 90, 99, 100]
    print(f"waves {len(a)}  kernel span {T:.1f} us")
    print("start us pct", dict(zip(q, np.percentile(start, q).round(1))))
    print("end   us pct", dict(zip(q, np.percentile(end, q).round(1))))
    print("tiles/wave pct", dict(zip(q, np.percentile(a[:, 2], q).round(1))))
    print(f"busy fraction {np.mean(end - start) / T:.3f}")


if __name__ == "__main__":
    main()
