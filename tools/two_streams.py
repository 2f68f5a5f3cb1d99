#!/usr/bin/env python3
"""Concurrency probe (diagnostic): does a second, independent pipeline on a
second HIP stream raise throughput (the resolve of one batch co-running with
the traversal of another)?  Two scene replicas on device 0, 36-frame orbit."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene
    tris, _ = sponza_scene()
    A = rt.Scene(tris, "bsah", 8).upload([0])
    B = rt.Scene(tris, "bsah", 8).upload([0])
    W, H = 1920, 1080
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(36)]
    bufs = [torch.empty((36, H, W), dtype=torch.int32, device="cuda:0") for _ in range(2)]
    rgbs = [torch.empty((36, H, W, 3), dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def one(scene, k, cam_list, stream):
        scene.render_batch_device(0, cam_list, W, H, 0, 1, H, hit_id=bufs[k].data_ptr(), rgb=rgbs[k].data_ptr(),
                                  stream=stream.cuda_stream)

    for _ in range(2):
        one(A, 0, cams, s1)
        one(B, 1, cams, s2)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        one(A, 0, cams, s1)
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(reps):
        one(A, 0, cams[:18], s1)
        one(B, 1, cams[18:], s2)
    torch.cuda.synchronize()
    t2 = time.perf_counter() - t0
    rays = reps * 36 * W * H
    print(f"one stream {rays / t1 / 1e6:.0f} Mrays/s, two streams {rays / t2 / 1e6:.0f} Mrays/s")


if __name__ == "__main__":
    main()
