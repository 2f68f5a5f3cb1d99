#!/usr/bin/env python3
"""First-launch cost of the headline kernel in a fresh process (VERDICT r5
item 3: does the traversal kernel's private segment cost a cold launch?).

    python tools/cold_launch.py [--reps N] [--out FILE]

Each repetition is a child process (the library under test is RT_LIB, or the
shipped one) that builds the sponza proxy scene, uploads it, and times with
host clocks around a device synchronise:
  * the first rt_render_batch_device call of the 36-pose orbit (the HIP
    runtime backs the kernel's private segment on its first dispatch), the
    second and the third;
  * then the first and second rt_render_frame (the drop-in path, one pose).
Prints one JSON line per process and a summary (medians).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, {root!r})
import torch
import raytracingdemo_amd as rt
from raytracingdemo_amd.scenes import sponza_scene
tris, label = sponza_scene()
s = rt.Scene(tris, "bsah", 8).upload([0])
W, H = 1920, 1080
path = rt.CameraPath(rt.scene_center(tris), 36)
cams = [path.circular_path(f) for f in range(36)]
ids = torch.empty((36, H, W), dtype=torch.int32, device="cuda:0")
dist = torch.empty((36, H, W), dtype=torch.float64, device="cuda:0")
rgb = torch.empty((36, H, W, 3), dtype=torch.uint8, device="cuda:0")
cnt = torch.zeros(36, dtype=torch.int64, device="cuda:0")
torch.cuda.synchronize()
st = torch.cuda.current_stream().cuda_stream
out = {{}}
for k in range(3):
    t0 = time.perf_counter()
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ids.data_ptr(), dist=dist.data_ptr(), rgb=rgb.data_ptr(),
                          hit_count=cnt.data_ptr(), stream=st, counts_store=True)
    torch.cuda.synchronize()
    out[f"batch{{k}}_ms"] = (time.perf_counter() - t0) * 1e3
g = None
for k in range(2):
    t0 = time.perf_counter()
    g = s.calculate_screen(*cams[k], W, H, want=("hit_id", "pos"), out=g)
    out[f"frame{{k}}_ms"] = (time.perf_counter() - t0) * 1e3
print("COLD", json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for _ in range(a.reps):
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            raise SystemExit(r.returncode)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("COLD ")][-1]
        d = json.loads(line[5:])
        rows.append(d)
        print(json.dumps(d), flush=True)
    summ = {k: round(statistics.median(r[k] for r in rows), 3) for k in rows[0]}
    res = {"lib": os.environ.get("RT_LIB") or "shipped", "reps": a.reps, "median_ms": summ}
    print("SUMMARY", json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"runs": rows, **res}, fh, indent=1)


if __name__ == "__main__":
    main()
