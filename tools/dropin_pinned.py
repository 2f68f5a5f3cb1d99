"""Drop-in frame call (rt_render_frame) into pageable vs pinned host arrays
(diagnostic for INTEGRATION.md §2: does the binding gain from hipHostMalloc'd
ray-hit buffers?).  Sponza proxy, 1080p, the 36-pose orbit, hit id + position."""
import time

import numpy as np
import torch

import raytracingdemo_amd as rt
from raytracingdemo_amd.scenes import sponza_scene

W, H = 1920, 1080
tris, _ = sponza_scene()
s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
path = rt.CameraPath(rt.scene_center(tris), 36)
cams = [path.circular_path(f) for f in range(36)]
npx = W * H


def run(out):
    for p, d in cams[:2]:
        s.calculate_screen(p, d, W, H, out=out)
    t0 = time.perf_counter()
    for p, d in cams:
        s.calculate_screen(p, d, W, H, out=out)
    return (time.perf_counter() - t0) / len(cams) * 1e3


for want in (("hit_id", "pos"), ("hit_id", "dist", "rgb"), ("rgb",)):
    page = {k: None for k in ("hit_id", "dist", "pos", "rgb")}
    pin = dict(page)
    shapes = {"hit_id": ((npx,), np.uint32, torch.int32), "dist": ((npx,), np.float64, torch.float64),
              "pos": ((npx, 3), np.float64, torch.float64), "rgb": ((npx, 3), np.uint8, torch.uint8)}
    keep = []
    for k in want:
        shp, nd, td = shapes[k]
        page[k] = np.empty(shp, nd)
        t = torch.empty(shp, dtype=td, pin_memory=True)
        keep.append(t)
        pin[k] = t.numpy().view(nd)
    a, b = run(page), run(pin)
    print(f"{'+'.join(want):18s} pageable {a:.3f} ms/frame ({npx / a / 1e3:.0f} Mrays/s)   "
          f"pinned {b:.3f} ms/frame ({npx / b / 1e3:.0f} Mrays/s)", flush=True)
