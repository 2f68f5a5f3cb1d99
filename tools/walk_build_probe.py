#!/usr/bin/env python3
"""Times the device walk-tree build on the sponza proxy (several builds in one
process) next to the host build: python tools/walk_build_probe.py [reps]."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracingdemo_amd as rt  # noqa: E402
from raytracingdemo_amd.scenes import sponza_proxy_triangles  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.cuda.set_device(0)
tris = sponza_proxy_triangles()
for k in range(reps):
    t0 = time.perf_counter()
    s = rt.Scene(tris, "bsah", 8, walk_device=0)
    t1 = time.perf_counter()
    print(f"device build {k}: total {1e3 * (t1 - t0):.1f} ms", {a: round(b, 1) for a, b in s.build_times().items()},
          flush=True)
h = rt.Scene(tris, "bsah", 8)
print("host build:", {a: round(b, 1) for a, b in h.build_times().items()}, flush=True)
