#!/usr/bin/env python3
"""Exchange-beside-render probe (diagnostic, one GPU): can a step's payload
leave the device while the next step renders?

Renders the per-GPU work of an N-GPU headline run (shard 0 of N of the
36-pose 1080p orbit, `rt_render_shard_device`) on two alternating streams,
as bench.py does, and after each render issues that step's payload copy
(the rgb framebuffers, 3 B per pixel: bench.py's `ship()` payload, 28 MB at
N = 8) on a high-priority side stream.  Modes:

  none   no copy (the render rate alone)
  blit   device-to-device copy (torch copy_: a copy KERNEL, which needs CU
         slots — as RCCL's gather kernels do)
  sdma   device-to-host copy into pinned memory (the copy ENGINE: no CU slots;
         but PCIe-bound at ~53 GB/s, so no stand-in for a peer copy over xGMI)
  rccl   a one-rank RCCL gather through torch.distributed (RCCL's own
         kernels, on its high-priority stream: do they find a slot?)

For each mode: the step time over the timed steps, and per step the delay
from the render's end to the copy's end (HIP events).  RT_PACKET_BLOCKS_PER_CU
(read by the library at upload) leaves block slots free on every CU for the
blit mode.  Prints one JSON line per mode.

    python tools/exchange_probe.py [--shard-of 8] [--steps 200] [--modes none,blit,sdma]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--modes", default="none,blit,sdma")
    a = ap.parse_args()
    import torch

    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import sponza_scene

    tris, label = sponza_scene()
    scene = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    W, H, F, G = 1920, 1080, 36, a.shard_of
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(F)]
    rows = rt.shard_height(H, G, 0)
    dev = torch.device("cuda", 0)
    NB = 2
    ids = [torch.empty((F, rows, W), dtype=torch.int32, device=dev) for _ in range(NB)]
    dists = [torch.empty((F, rows, W), dtype=torch.float64, device=dev) for _ in range(NB)]
    rgb = [torch.empty((F, rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(NB)]
    cnt = [torch.zeros((F,), dtype=torch.int64, device=dev) for _ in range(NB)]
    dst_dev = [torch.empty_like(rgb[0]) for _ in range(NB)]
    dst_host = [torch.empty(rgb[0].shape, dtype=torch.uint8, pin_memory=True) for _ in range(NB)]
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    side = torch.cuda.Stream(dev, priority=-1)

    def render(b):
        scene.render_shard_device(0, cams, W, H, 0, G, hit_id=ids[b].data_ptr(), dist=dists[b].data_ptr(),
                                  rgb=rgb[b].data_ptr(), hit_count=cnt[b].data_ptr(), stream=streams[b].cuda_stream)

    dist = None
    if "rccl" in a.modes:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29611")
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, pg_options=opts)
    for mode in a.modes.split(","):
        shipped = [None] * NB
        delays = []
        evs = []

        def step(k, timed):
            b = k % NB
            with torch.cuda.stream(streams[b]):
                if shipped[b] is not None:
                    streams[b].wait_event(shipped[b])  # the copy has read the buffer
                render(b)
                e_r = torch.cuda.Event(enable_timing=True)
                e_r.record(streams[b])
            if mode == "none":
                shipped[b] = None
                return
            side.wait_stream(streams[b])
            with torch.cuda.stream(side):
                if mode == "rccl":
                    w = dist.gather(rgb[b], [dst_dev[b]], dst=0, async_op=True)
                    w.wait()
                elif mode == "blit":
                    dst_dev[b].copy_(rgb[b])
                else:
                    dst_host[b].copy_(rgb[b], non_blocking=True)
                e_c = torch.cuda.Event(enable_timing=True)
                e_c.record(side)
            shipped[b] = e_c
            if timed:
                evs.append((e_r, e_c))

        for k in range(20):  # warm-up and clock settle
            step(k, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(k, True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        delays = [r.elapsed_time(c) for r, c in evs]
        out = {"mode": mode, "shard_of": G, "packet_blocks_per_cu": os.environ.get("RT_PACKET_BLOCKS_PER_CU", "max"),
               "payload_MB": round(rgb[0].numel() / 1e6, 2), "steps": a.steps,
               "ms_per_step": round(el / a.steps * 1e3, 4),
               "Mrays_per_s": round(a.steps * F * rows * W / el / 1e6, 1)}
        if delays:
            out["copy_done_after_render_ms"] = {"median": round(statistics.median(delays), 4),
                                                "p10": round(sorted(delays)[len(delays) // 10], 4),
                                                "p90": round(sorted(delays)[len(delays) * 9 // 10], 4)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
