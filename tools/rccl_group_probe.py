#!/usr/bin/env python3
"""Runs the in-library RCCL branch of render_group (rt_api.cpp) on one GPU:
RT_GROUP_RCCL=1 gives a one-device scene a one-rank communicator, so
rt_render_batch_multi renders its shard, gathers it with ncclGather (group
start/end) into the root buffer and de-interleaves it.  Checked against the
one-device render; run under `rocprofv3 --kernel-trace` to see the RCCL kernel
between the shard's render and k_deinterleave (profiles/r03_rccl_*)."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import raytracingdemo_amd as rt
    from conftest import golden_scene

    tris = golden_scene("stanford-bunny.obj")
    s = rt.Scene(tris, "bsah", 8).upload([0])
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(6)]
    W, H, F = 640, 360, len(cams)
    st = torch.cuda.current_stream().cuda_stream
    ref_id = torch.empty(F * H * W, dtype=torch.int32, device="cuda:0")
    ref_rgb = torch.empty(F * H * W * 3, dtype=torch.uint8, device="cuda:0")
    ref_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ref_id.data_ptr(), rgb=ref_rgb.data_ptr(),
                          hit_count=ref_cnt.data_ptr(), stream=st)
    os.environ["RT_GROUP_RCCL"] = "1"
    for it in range(3):
        g_id = torch.full_like(ref_id, 7)
        g_rgb = torch.full_like(ref_rgb, 7)
        g_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
        s.render_batch_multi(cams, W, H, hit_id=g_id.data_ptr(), rgb=g_rgb.data_ptr(), hit_count=g_cnt.data_ptr(),
                             stream=st)
        torch.cuda.synchronize()
        ok = torch.equal(g_id, ref_id) and torch.equal(g_rgb, ref_rgb) and torch.equal(g_cnt, ref_cnt)
        print(f"rccl group call {it}: {'equal' if ok else 'DIFFERENT'} to the one-device render "
              f"({int(g_cnt.sum())} hits over {F} poses)", flush=True)
        if not ok:
            sys.exit(1)
    assert np.all(ref_cnt.cpu().numpy() > 0)


if __name__ == "__main__":
    main()
