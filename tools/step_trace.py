"""Per-step timeline of the headline workload (36 poses of the sponza proxy at
1920x1080 per step, one library call each), to see how the step time moves
with the GPU's clock after start: HIP events around every step, printed as
one JSON line of per-step milliseconds.  Not a measurement of record; it
sizes bench.py's warm-up.

    python tools/step_trace.py [--steps 200] [--shard-of 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--shard-of", type=int, default=1)
    a = p.parse_args()
    import torch

    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene
    from raytracingdemo_amd.shards import shard_rows

    dev = torch.device("cuda", 0)
    tris, label = sponza_scene()
    scene = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    W, H, F = 1920, 1080, 36
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(F)]
    rows = len(shard_rows(0, a.shard_of, H))
    ids = torch.empty((F, rows, W), dtype=torch.int32, device=dev)
    rgb = torch.empty((F, rows, W, 3), dtype=torch.uint8, device=dev)
    cnt = torch.zeros((F,), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev[0].record(st)
    for k in range(a.steps):
        scene.render_shard_device(0, cams, W, H, 0, a.shard_of, hit_id=ids.data_ptr(), rgb=rgb.data_ptr(),
                                  hit_count=cnt.data_ptr(), stream=st.cuda_stream)
        ev[k + 1].record(st)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = [round(ev[k].elapsed_time(ev[k + 1]), 4) for k in range(a.steps)]
    print(json.dumps({"workload": f"{label} 1920x1080 x36 poses, shard 0 of {a.shard_of}", "steps": a.steps,
                      "wall_s": round(wall, 3), "ms_per_step": ms}))


if __name__ == "__main__":
    main()
