#!/usr/bin/env python3
"""Where the headline kernel's time goes, by phase of a tile.

Needs a measurement build of the library with RT_PROFILE=1
(`make -C raytracingdemo_amd/csrc variant V=prof VFLAGS=-DRT_PROFILE=1`,
selected with RT_LIB=...): the timed k_trace_packet then adds the shader-clock
cycles of each tile's phases to counters 18-23 (packet_kernel.h), read here
with rt_diag_raw after the bench workload (sponza proxy, 1920x1080, the
36-pose orbit in one launch).  Cycles are per wave, summed over all tiles; the
shares are what matter (s_memtime reads cost some overlap themselves).

    RT_LIB=.../librtmi355x_prof.so python tools/phase_profile.py [--launches 5] [--out f.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    import raytracingdemo_amd as rt
    from raytracingdemo_amd import _native as N
    from raytracingdemo_amd.scenes import sponza_proxy_triangles

    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(36)]
    W, H, F = 1920, 1080, 36
    ids = torch.empty((F, H, W), dtype=torch.int32, device="cuda:0")
    dist = torch.empty((F, H, W), dtype=torch.float64, device="cuda:0")
    rgb = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
    cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream

    def launch():
        s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ids.data_ptr(), dist=dist.data_ptr(),
                              rgb=rgb.data_ptr(), hit_count=cnt.data_ptr(), stream=st, timing=True)

    launch()
    torch.cuda.synchronize()
    s.frame_stats(0, reset=True)
    for _ in range(a.launches):
        launch()
    torch.cuda.synchronize()
    raw = (C.c_uint64 * 24)()
    N.check(N.lib().rt_diag_raw(s.handle, 0, raw, 24))
    fs = s.frame_stats(0, reset=True)
    c = np.array(list(raw), dtype=np.float64)
    tiles = c[22]
    if tiles == 0:
        raise SystemExit("no profile counters: is RT_LIB a RT_PROFILE=1 build?")
    phases = {"setup": c[18], "node_steps": c[19], "leaf_steps": c[20], "resolve_and_stores": c[21]}
    total = c[23]
    res = {"tiles": int(tiles), "cycles_per_tile": {k: round(v / tiles, 1) for k, v in phases.items()},
           "cycles_per_tile_total": round(total / tiles, 1),
           "share": {k: round(v / total, 4) for k, v in phases.items()},
           "kernel_ms_avg": round(fs["trace_ms"] / max(fs["timed_launches"], 1), 4),
           "workload": "sponza proxy 1920x1080, 36-pose orbit per launch, RT_PROFILE build",
           "lib": os.environ.get("RT_LIB", "")}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
