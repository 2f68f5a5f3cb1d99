#!/usr/bin/env python3
"""Per-ray work of the REFERENCE's traversal (StackBVH::traverse,
src/stack_bvh.hpp:611-644: every box popped is tested, children of a hit box
are pushed, every leaf triangle of a hit leaf is tested) on the headline scene,
next to SURVEY.md §8(a) a1's probes of the published models — how hard the
sponza proxy is compared with the scenes the reference was measured on.

Counts come from the oracle's literal traversal (oracle/rt_oracle.cpp
traverse(): box tests, box hits, triangle tests), on the same bsah-k tree the
reference builds.  Writes profiles/scene_difficulty.json (read by bench.py).

    python tools/scene_difficulty.py [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def per_ray(b, cams, W, H, threads):
    bt = bh = tt = rays = hits = 0
    for pos, d in cams:
        o = b.render(pos, d, W, H, threads=threads, want=("id",))
        c = o["counters"]
        bt, bh, tt = bt + c[0], bh + c[1], tt + c[2]
        rays += W * H
        hits += o["hits"]
    return {"box_tests": round(bt / rays, 3), "box_hits": round(bh / rays, 3), "box_misses": round((bt - bh) / rays, 3),
            "tri_tests": round(tt / rays, 3), "hit_fraction": round(hits / rays, 4), "rays": rays}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    import pyoracle
    import raytracingdemo_amd as rt
    from conftest import golden_scene
    from raytracingdemo_amd.scenes import sponza_proxy_triangles

    o = pyoracle.Oracle()
    out = {}
    tris = sponza_proxy_triangles()
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (0, 9, 18, 27)]
    b = o.bvh(tris, "bsah", 8)
    r = per_ray(b, cams, 1920, 1080, a.threads)
    r["sample"] = "frames 0, 9, 18, 27 of the orbit at 1920x1080, bsah-8"
    out["sponza-proxy (procedural, 262267 tris)|bsah-8"] = r
    # the probes SURVEY.md §8(a) a1 quotes (500x500, frame 0): bunny BVH8
    # 4.1 + 21.5 box tests and 3.4 triangle tests per ray, teapot 4.2 + 19.0
    # and 4.0 — the same convention reproduced here
    probes = {}
    for model in ("stanford-bunny.obj", "teapot.obj"):
        t = golden_scene(model)
        c = rt.CameraPath(rt.scene_center(t), 36).circular_path(0)
        probes[model] = per_ray(o.bvh(t, "bsah", 8), [c], 500, 500, a.threads)
        probes[model]["sample"] = "frame 0 at 500x500, bsah-8"
    for v in out.values():
        v["reference_probes"] = probes
        v["note"] = ("per ray: box_hits = boxes the reference enters (SURVEY a1's positive box tests), "
                     "box_misses = boxes it tests and rejects, tri_tests = Moller-Trumbore calls")
    dst = os.path.join(ROOT, "profiles", "scene_difficulty.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
