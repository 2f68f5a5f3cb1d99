#!/usr/bin/env python3
"""Headline benchmark: Mrays/s of primary rays (1 spp) on Sponza 1920x1080,
BVH8 (bsah-8 k-way), plus the HBM-roofline fraction of the traversal kernel and
a CPU baseline (the reference's own traversal, compiled, all host cores used).

A *step* is one pass of the reference's camera orbit (runTest's 36-frame path,
src/main.cpp:234-281): every frame is ray generation + traversal + exact
resolve + shading on the GPU, bands of 8 image rows interleaved over the N
GPUs (band b on rank b mod N: rt_render_shard_device), followed by one RCCL
gather of the step's framebuffers (rgb) and hit
counts to rank 0 and the de-interleave there, on a side stream that overlaps
the next step's render.  Total work per step is fixed (strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Sponza's geometry is absent from the reference (.MISSING_LARGE_BLOBS:1): the
scene is the procedural 262,267-triangle proxy (raytracingdemo_amd.scenes)
unless RT_SPONZA_OBJ points at a real sponza.obj.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec (primary, 1spp) on Sponza 1920×1080; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# what `traffic` counts (tools/pmc_traffic.py): the L2's memory-side requests
# (FETCH_SIZE with the gfx950 unit correction per access type, + WRITE_SIZE);
# Infinity-Cache (MALL) hits are included, so it is L2-miss / fabric traffic,
# an upper bound of the HBM bytes
TRAFFIC_COUNTS = ("L2-miss (fabric) bytes: FETCH_SIZE (x2 for vector reads, calibrated) + WRITE_SIZE; "
                  "Infinity-Cache hits included, so an upper bound of HBM bytes")
TRI32_BYTES = 48       # fp32 pre-filter record (v0, e1, e2 + 3 bounds)
TRI64_BYTES = 128      # fp64 record (v0, e1, e2, normal, id, leaf, leaf box) per exact test
MT64_BYTES = 72        # its Moller-Trumbore part (v0, e1, e2) per exact test (fused resolve)
WIN_BYTES = 56         # the winner's normal, {id, leaf} and leaf box, once per hit pixel
CHAIN_BYTES = 52       # fp64 box (48 B) + parent (4 B) per re-verified ancestor
OUT_BYTES = 15         # u32 hit-id + f64 distance + 3 B rgb written per ray
CAND_BYTES = 8         # one candidate entry {triangle, t bound} handed to the resolve kernel
SAMPLE_BYTES = 37      # spp > 1, fused: u32 hit-id + f64 distance + the sample's f64 colour + status byte
PACKED_SAMPLE_BYTES = 12  # spp 4 / 16, fused and packed (one wave holds a pixel's samples): hit-id + distance
SETTLE_S = 0.1         # untimed render-only steps after the W warm-up steps: at least this much GPU work


def host_cores():
    """CPUs this process may use: the cgroup CPU quota (cpu.max) and the
    affinity mask, next to what the machine reports (nproc honours
    OMP_NUM_THREADS; std::thread::hardware_concurrency = os.cpu_count())."""
    info = {"hardware_concurrency": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        import subprocess
        info["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
            info["cgroup_cpu_max"] = f"{q} {per}"
    except (OSError, ValueError):
        pass
    usable = info["affinity"]
    if quota:
        usable = min(usable, max(1, int(quota)))
    info["usable"] = usable
    return info


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--frames", type=int, default=None, help="camera-path frames per step (runTest: 36; paths: 1)")
    p.add_argument("--width", type=int, default=None, help="default 1920 (paths: 3840)")
    p.add_argument("--height", type=int, default=None, help="default 1080 (paths: 2160)")
    p.add_argument("--paths", action="store_true",
                   help="config c5: diffuse path tracing (secondary rays), 16 spp x (1 + 4 bounces) by default")
    p.add_argument("--bounces", type=int, default=4, help="paths: secondary bounces per sample")
    p.add_argument("--pipeline", default=os.environ.get("RT_PATHS", "auto"), choices=["auto", "queue", "mega"],
                   help="paths: the queued tracer (compacted per-segment queues) or the megakernel (sets RT_PATHS "
                        "for the library); auto: the library's default (queued with occlusion rays or packet primaries "
                        "(8-wide tree, spp 4 or 16), else mega)")
    p.add_argument("--no-shadow", action="store_true",
                   help="paths: no occlusion rays toward the head-light at the bounce vertices (RT_FLAG_SHADOW)")
    p.add_argument("--scene", default="sponza", choices=["sponza", "armadillo"],
                   help="sponza: configs c4/c5 (the headline; proxy unless RT_SPONZA_OBJ); "
                        "armadillo: config c3 (needs RT_ARMADILLO_OBJ, the geometry is stripped from the reference)")
    p.add_argument("--algo", default="bsah")
    p.add_argument("--k", type=int, default=8)
    p.add_argument("--mode", default="exact", choices=["exact", "fp64"])
    p.add_argument("--spp", type=int, default=None, help="samples per pixel: stratified n*n for primary rays "
                                                         "(config c4: 4; headline: 1), paths default 16")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-dropin", action="store_true", help="skip the rt_render_frame (drop-in path) rate")
    p.add_argument("--no-overlap", action="store_true",
                   help="issue every step on one stream (no overlap of consecutive steps' launches)")
    p.add_argument("--shard-of", type=int, default=1,
                   help="diagnostic (one process): render only shard 0 of N interleaved row shards — the per-GPU "
                        "work of an N-rank run without its gather; not the headline")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="committed rocprofv3 PMC summary supplying roofline.traffic")
    p.add_argument("--key-out", default="", help="write this run's workload key (for tools/pmc_traffic.py)")
    a = p.parse_args()
    a.frames = a.frames if a.frames is not None else (1 if a.paths else 36)
    a.width = a.width if a.width is not None else (3840 if a.paths else 1920)
    a.height = a.height if a.height is not None else (2160 if a.paths else 1080)
    a.spp = a.spp if a.spp is not None else (16 if a.paths else 1)
    return a


def cpu_baseline(tris, algo, k, cams, W, H, target_s, gpu=None):
    """Reference traversal (oracle/_ref: the reference's own headers compiled -O3,
    OpenMP over pixel columns; the timed scope of runTest, src/main.cpp:253-255)
    or, without it, the oracle restatement, in two legs: every host core this
    process may use (the cgroup quota on the GPU box) and one core.  Bounded
    samples: whole frames of the same camera orbit until ~target_s of CPU time
    (all cores), ~target_s / 3 (one core: whole rows, a frame is ~3 s there).

    gpu: the timed step's outputs (numpy hit ids, distances, colours and hit
    counts per pose, N = 1): every whole frame the reference renders here is
    compared with them — hit mask, |hit - o| from its fp64 hit point (the
    stack_bvh.hpp:631 expression), PPM bytes and hit count."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    host = host_cores()
    threads = int(os.environ.get("RT_CPU_THREADS", host["usable"]))
    if pyoracle.Reference.available():
        lib, kind = pyoracle.Reference(), "reference"
    else:
        lib, kind = pyoracle.Oracle(), "port"
    b = lib.bvh(tris, algo, k)
    frames, rays, spent = 0, 0, 0.0
    check = {"frames": 0, "pixels": 0, "hit_mask_diff": 0, "dist_diff": 0, "rgb_diff": 0, "count_diff": 0}
    while spent < target_s and frames < len(cams) * 4:
        f = frames % len(cams)
        pos, d = cams[f]
        t0 = time.perf_counter()
        o = b.render(pos, d, W, H, threads=threads)
        spent += time.perf_counter() - t0
        frames += 1
        rays += W * H
        if gpu is not None and frames <= len(cams):  # (outside the timed CPU work)
            hit = o["hit"] if "hit" in o else o["id"] >= 0
            g_hit = gpu["ids"][f] != -1
            p = np.asarray(pos, dtype=np.float64)
            dx, dy, dz = (o["pos"][:, a] - p[a] for a in range(3))
            rdist = np.sqrt(dx * dx + dy * dy + dz * dz)
            check["frames"] += 1
            check["pixels"] += W * H
            check["hit_mask_diff"] += int(np.count_nonzero(hit != g_hit))
            both = hit & g_hit
            check["dist_diff"] += int(np.count_nonzero(rdist[both] != gpu["dist"][f][both]))
            check["rgb_diff"] += int(np.count_nonzero(np.any(o["rgb"] != gpu["rgb"][f], axis=1)))
            check["count_diff"] += int(o["hits"] != int(gpu["cnt"][f]))
    # one core: bands of 60 rows spread over the orbit's frames
    rows1, spent1, f1 = 0, 0.0, 0
    while spent1 < target_s / 3 and f1 < len(cams) * (H // 60):
        pos, d = cams[f1 % len(cams)]
        row0 = (f1 * 7 * 60) % (H - 60 + 1)
        t0 = time.perf_counter()
        b.render(pos, d, W, H, row0=row0, nrows=60, threads=1)
        spent1 += time.perf_counter() - t0
        rows1 += 60
        f1 += 1
    one = rows1 * W / spent1 / 1e6
    return {"value": round(rays / spent / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": kind,
            "sample": f"{frames} full {W}x{H} frames of the same camera orbit ({rays} rays, {spent:.1f} s), "
                      f"same scene and {algo}-{k} tree, reference traversal semantics (no culling)",
            "all_cores": {"value": round(rays / spent / 1e6, 4), "cores": threads},
            "one_core": {"value": round(one, 4), "cores": 1,
                         "sample": f"{f1} bands of 60 rows x {W} px over the orbit ({rows1 * W} rays, {spent1:.1f} s)"},
            "host": host,
            **({"verified_timed_frames": dict(check, equal=not any(v for kk, v in check.items()
                                                                     if kk.endswith("_diff")))}
               if gpu is not None else {}),
            "published_O0": {"value": None, "note": "no published Sponza figure for the current code; the only "
                             "Sponza datum is an older-code run (testruns_2025_12_25/testrun_47: 105.58 s mean per "
                             "500x500 frame, 0.0024 Mrays/s, -O0, 1 core; not comparable). Published -O0 1-core "
                             "bsah-8 figures of the other models: 0.149-0.200 Mrays/s (BASELINE.md §1)"}}


def scene_difficulty(label, algo, k):
    """The reference's own per-ray work on this scene (oracle traversal
    counters over sampled frames; tools/scene_difficulty.py writes the
    committed summary), next to SURVEY.md §8(a) a1's bunny and teapot probes."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "scene_difficulty.json")))
    except (OSError, ValueError):
        return None
    key = f"{label}|{algo}-{k}"
    return d.get(key)


def rank_problems(table, backend, pg_size, world, gpus, rehearse):
    """What is wrong with an N-rank run, from every rank's [rank, local rank,
    device ordinal, PCI bus] row (rank order) and the process group's backend
    and size; [] when it is what --gpus asks for."""
    ordinals = [r[2] for r in table]
    problems = []
    if pg_size != gpus or world != gpus or len(table) != gpus:
        problems.append(f"process group size {pg_size} / WORLD_SIZE {world} / {len(table)} rows != --gpus {gpus}")
    if [r[0] for r in table] != list(range(len(table))):
        problems.append(f"ranks {[r[0] for r in table]}")
    if not rehearse:
        if backend != "nccl":
            problems.append(f"backend {backend}, not nccl (RCCL)")
        if len(set(ordinals)) != len(table) or len(set((r[3], r[2]) for r in table)) != len(table):
            problems.append(f"device ordinals {ordinals} (bus {[r[3] for r in table]}) not one per rank")
    return problems


def rank_facts(a, world, rank, local, dev, coll, rehearse):
    """Self-check of an N-rank run, before any timing: the
    process group's size and backend, every rank's device ordinal and PCI bus
    as the ranks themselves report them (all_gather over the same communicator
    that carries the frames).  Any disagreement with --gpus ends the run with
    exit status 1 on every rank (rehearsals: every rank on device 0 over gloo,
    by design)."""
    import torch
    import torch.distributed as dist
    backend = str(dist.get_backend())
    pg_size = dist.get_world_size()
    props = torch.cuda.get_device_properties(dev)
    bus = int(getattr(props, "pci_bus_id", -1))
    me = torch.tensor([rank, local, torch.cuda.current_device(), bus], dtype=torch.int64, device=dev)
    allv = [coll(torch.empty_like(me)) for _ in range(world)]
    dist.all_gather(allv, coll(me))
    table = [[int(x) for x in v.tolist()] for v in allv]
    problems = rank_problems(table, backend, pg_size, world, a.gpus, rehearse)
    facts = {"world_size": world, "process_group_size": pg_size, "backend": backend,
             "rccl": backend == "nccl", "device_ordinals": [r[2] for r in table], "pci_bus": [r[3] for r in table],
             "verified": not problems}
    if problems:
        if rank == 0:
            print(json.dumps({"error": "multi-rank self-check failed", "problems": problems, "ranks": facts}),
                  flush=True)
        dist.destroy_process_group()
        raise SystemExit(1)
    return facts


def run_paths(a, scene, tris, label, world, rank, local, dev, coll, rehearse, ranks=None):
    """Config c5: diffuse path tracing of primary + secondary rays (rt_render_paths_device).
    A step is one pose of the orbit (step k: frame k % 36), every rank tracing its
    interleaved rows, then one RCCL gather of the colours to rank 0, which
    de-interleaves.  value = W*H*spp*(1 + bounces) / time (SURVEY.md §8(d)'s
    nominal c5 ray count); segments actually traced are reported beside it."""
    import torch
    import torch.distributed as dist

    import raytracingdemo_amd as rt
    from raytracingdemo_amd.shards import gather_frames, rows_per_rank, shard_rows

    W, H, S, B, F = a.width, a.height, a.spp, a.bounces, a.frames
    shadow = not a.no_shadow
    if a.pipeline == "auto":  # the library's default (rt_api.cpp path_pipe)
        os.environ.pop("RT_PATHS", None)
        a.pipeline = "queue" if shadow or (S in (4, 16) and a.k == 8) else "mega"
    else:
        os.environ["RT_PATHS"] = a.pipeline  # (read by the library per call)
    queued = a.pipeline == "queue"
    # occlusion-ray mode (render.hip queued_shadow_mode): per lane where the
    # vertex is shaded (the megakernel; the queued pipeline with
    # RT_SHADOW_RAYS=lane), or queued: from records per lane
    # (RT_SHADOW_RAYS=rec) or sorted and walked by the wave (the queued
    # pipeline's default)
    sh_env = os.environ.get("RT_SHADOW_RAYS", "")[:1]
    shadow_kind = None if not shadow else ("records" if queued and sh_env == "r" else
                                           "inline" if not queued or sh_env == "l" else "binned")
    path = rt.CameraPath(rt.scene_center(tris), 36)
    rows = rows_per_rank(H, world, band=1)  # the paths kernel takes single interleaved rows
    my_rows = len(shard_rows(rank, world, H, band=1))
    rgb = torch.zeros((1, rows, W, 3), dtype=torch.uint8, device=dev)
    cnt = torch.zeros((1,), dtype=torch.int64, device=dev)
    gather_rgb = coll(rgb).new_empty((world,) + tuple(rgb.shape)) if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream(dev)

    def render(k, timing=False, count=False):
        pos, d = path.circular_path(k % 36)
        for f in range(F):
            scene.render_paths_device(local, pos, d, W, H, rank, world, my_rows, frame=k % 36, spp=S, bounces=B,
                                      rgb=rgb.data_ptr(), hit_count=cnt.data_ptr(), stream=stream.cuda_stream,
                                      timing=timing, count=count, shadow=shadow, counts_store=True)

    def step(k, timing=False, count=False):
        render(k, timing=timing, count=count)
        if world > 1:
            return gather_frames(coll(rgb), H, world, rank, out=gather_rgb, band=1)
        return rgb

    render(0, count=True)  # counting pass: segments traced (outside timing)
    torch.cuda.synchronize(dev)
    cs = scene.frame_stats(local, reset=True)
    segs_per_pose = cs["rays"] / F
    sh_per_pose = cs["shadow_rays"] / F  # occlusion rays (0 without RT_FLAG_SHADOW)
    if shadow_kind == "binned" and cs["shadow_rays"] and not cs["shadow_wave_nodes"]:
        shadow_kind = "inline"  # (a walk tree deeper than the binned walk's stack: per lane)
    # algorithmic bytes of one pose (the counting pass, W = 8): per segment the
    # lane's own node steps on the 96-B quantised nodes (walk_tree.cpp
    # quantize_wide8), 48-B fp32 triangle records through the pre-filter,
    # 72-B fp64 Moller-Trumbore records, 52 B per ancestor-chain check and the
    # winner's 56-B record; 3 B of colour per pixel
    # (primary segments walked by the wave, path_kernel.h wave_walk: 256-B
    # nodes and 48-B triangle records once per wave)
    alg_walk = (cs["node_fetches"] * 96 + cs["wave_nodes"] * 256 + cs["wave_tris"] * 48 + cs["tri_prefilter"] * 48
                + cs["tri_tests"] * 72 + cs["chain_checks"] * 52 + cs["rays"] * 56) / F + my_rows * W * 3
    alg_pose, alg_parts = alg_walk, {"walks_and_resolve": round(alg_walk)}
    if queued:
        # the queued pipeline's own traffic (queue_paths.h): every bounce ray's
        # 80-B queue entry written once and read once, every path's final
        # radiance written and read (24 B each way)
        samples = my_rows * W * S
        bounce_rays = (cs["rays"] / F) - samples
        q_bytes = bounce_rays * 160 + samples * 48
        alg_pose += q_bytes
        alg_parts["queues"] = round(q_bytes)
    if shadow:
        # occlusion rays: the walk's fetches — binned records walked by the
        # wave (256-B nodes, 48-B triangle records once per wave), else per
        # lane (96-B quantised nodes, 48-B fp32 records per lane) — plus, for
        # queued records, each 32-B record's trips (binned: the record and
        # its 4-B key written; the 3 sort passes of 7 bits (19-bit keys) move (key, record)
        # pairs: histogram reads of 4, 8 and 8 B, scatters of 4 -> 8, 8 -> 8
        # and 8 -> 8 B; the walk reads its pair and gathers the record = 140
        # B; per-lane records kernel: written and read) and the lit ones'
        # radiance read and written (48 B)
        sh_n = cs["shadow_rays"]
        sh_lit = sh_n - cs["shadow_occluded"]
        if shadow_kind == "binned":
            sh_bytes = sh_n * 140 + sh_lit * 48 + cs["shadow_wave_nodes"] * 256 + cs["shadow_wave_tris"] * 48
        else:
            sh_bytes = cs["shadow_lane_nodes"] * 96 + cs["shadow_lane_tris"] * 48
            if shadow_kind == "records":
                sh_bytes += sh_n * 64 + sh_lit * 48
        alg_pose += sh_bytes / F
        alg_parts["occlusion"] = round(sh_bytes / F)
    # The headline's convention, a record once per fetching wave instruction,
    # applied to the per-lane walks too (the per-lane figure
    # above is not comparable with the headline's): the lane walks' node
    # steps and triangle records counted once per distinct record among the
    # lanes of each wave step (render.hip wave_step_fetches), the fp64
    # records, queues and outputs as above.  None if the counting pass did
    # not fill the wave-distinct counters (a library without them).
    alg_wave = None
    if cs.get("lane_wave_nodes"):
        lane_bytes = (cs["node_fetches"] * 96 + cs["tri_prefilter"] * 48 +
                      (cs["shadow_lane_nodes"] * 96 + cs["shadow_lane_tris"] * 48 if shadow_kind != "binned" else 0))
        alg_wave = alg_pose + (cs["lane_wave_nodes"] * 96 + cs["lane_wave_tris"] * 48 - lane_bytes) / F
    # W warm-up steps, then render-only steps until SETTLE_S of GPU work (main())
    for w in range(a.warmup):
        step(w, timing=True)
    torch.cuda.synchronize(dev)
    settled = 0
    t_set = time.perf_counter()
    while time.perf_counter() - t_set < SETTLE_S:
        render(settled, timing=True)
        torch.cuda.synchronize(dev)
        settled += 1
    scene.frame_stats(local, reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k, timing=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ks = scene.frame_stats(local, reset=True)
    if world > 1:
        t = coll(torch.tensor([elapsed], dtype=torch.float64, device=dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        sg = coll(torch.tensor([segs_per_pose, sh_per_pose], dtype=torch.float64, device=dev))
        dist.all_reduce(sg, op=dist.ReduceOp.SUM)
        segs_per_pose, sh_per_pose = float(sg[0].item()), float(sg[1].item())
    nominal = a.steps * F * W * H * S * (1 + B)
    kernel_s = ks["trace_ms"] / max(ks["timed_launches"], 1) / 1e3
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu:
            # (the rows the CPU leg renders come from the last timed pose and
            # are compared with that pose's timed colours)
            k_last = (a.steps - 1) % 36
            cpu = paths_cpu_baseline(tris, a, path, W, H, S, B, shadow, pose=k_last,
                                     gpu_rgb=rgb[0].reshape(H, W, 3).cpu().numpy())
        key = (f"{label}|{W}x{H}|{a.algo}-{a.k}|paths|spp{S}|b{B}|n{world}" + ("|shadow" if shadow else "")
               + f"|{a.pipeline}")
        if a.key_out:
            with open(a.key_out, "w") as fh:
                fh.write(key + "\n")
        traffic = None
        try:
            pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_paths.json")))
            if pm.get("workload_key") == key:
                traffic = round(float(pm["hbm_bytes_per_launch"]))
        except (OSError, ValueError, KeyError):
            pass
        # frac counts bytes as the headline's does — a record once per
        # fetching wave instruction (alg_wave); the lane
        # walks counted per lane stay beside it (frac_lane_walks_per_lane)
        alg_frac = alg_wave if alg_wave else alg_pose
        achieved = alg_frac / kernel_s / 1e9 if kernel_s > 0 else 0.0
        achieved_lw = alg_pose / kernel_s / 1e9 if kernel_s > 0 else 0.0
        # the per-lane convention beside it: the primary segments' wave-walk
        # records counted once per lane (64) instead of once per wave; every
        # other walk here is per lane in both
        per_lane_pose = alg_pose + 63.0 * (cs["wave_nodes"] * 256 + cs["wave_tris"] * 48) / F
        achieved_pl = per_lane_pose / kernel_s / 1e9 if kernel_s > 0 else 0.0
        valu = None
        try:
            pv = json.load(open(os.path.join(ROOT, "profiles", "pmc_valu_paths.json")))
            if pv.get("workload_key") == key:
                valu = {"busy": pv["valu_busy"], "issue": issue_roofline(pv),
                        "wave_cycles_split": pv.get("wave_cycles_split"), "source": "profiles/pmc_valu_paths.json"}
        except (OSError, ValueError, KeyError):
            pass
        line = {
            # (the occlusion rays change the work per nominal ray: they are in
            # the metric's name, so a no-shadow line stays comparable with the
            # round-3 lines of the same name)
            "metric": f"Mrays/sec (primary + {B} diffuse bounces, {S}spp" + (" + head-light occlusion" if shadow else "")
                      + f") on Sponza {W}x{H}",
            "value": round(nominal / elapsed / 1e6, 2), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "settle_steps": settled,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32 traversal + f64 exact hits",
            "data": f"synthetic: {label}",
            "config": {"workload": f"{label}, {W}x{H}x{S}spp, 1 + {B} bounce segments per sample, diffuse paths, "
                                   f"{a.algo}-{a.k} reference tree, SAH walk tree, {F} pose(s) per step"
                                   + (", one head-light occlusion ray per bounce vertex" if shadow else ""),
                       "width": W, "height": H, "spp": S, "bounces": B, "frames_per_step": F,
                       "parallelism": f"image rows interleaved x{world}" + (" + RCCL gather" if world > 1 else ""),
                       **({"ranks": {**ranks, "gather_bytes_per_step": world * rows * W * 3 * F}} if ranks else {}),
                       **({"rehearsal_not_a_measurement": True} if rehearse else {})},
            "segments_traced_per_s_M": round(segs_per_pose * a.steps * F / elapsed / 1e6, 2),
            # every ray the pose traced: path segments plus occlusion rays
            "rays_traced_per_s_M": round((segs_per_pose + sh_per_pose) * a.steps * F / elapsed / 1e6, 2),
            "segments_per_sample": round(segs_per_pose / (W * H * S), 3),
            "pipeline": ("queued: wave-walked primaries, compacted per-segment bounce queues, per-lane bounce walks"
                         if queued else "megakernel (k_paths)"),
            "shadow": {"on": shadow, "mode": {"binned": "queued records, sorted by direction from the light, "
                                                     "walked by the wave (any hit)",
                                           "records": "queued records walked per lane (any hit)",
                                           "inline": "walked per lane where the vertex is shaded (any hit)",
                                           None: None}[shadow_kind], "rays_per_pose": round(cs["shadow_rays"] / F),
                       "occluded_per_pose": round(cs["shadow_occluded"] / F),
                       "rays_per_sample": round(cs["shadow_rays"] / F / (W * my_rows * S), 3),
                       "note": "one occlusion ray toward the head-light per bounce vertex (RT_FLAG_SHADOW); not "
                               "counted in value's nominal W*H*spp*(1+bounces)"},
            "kernel_ms_avg": round(ks["trace_ms"] / max(ks["timed_launches"], 1), 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "frac_convention": ("per wave instruction (the headline's): every walk's records once per "
                                             "fetching wave instruction" if alg_wave else
                                             "lane walks per lane (no wave-distinct counters in this library)"),
                         # the per-lane bounce and occlusion walks' records per lane
                         # (round 4-5's frac), and every walk per lane
                         "frac_lane_walks_per_lane": round(achieved_lw / HBM_PEAK_GBS, 4),
                         "alg_bytes_lane_walks_per_lane": round(alg_pose),
                         "frac_per_lane": round(achieved_pl / HBM_PEAK_GBS, 4),
                         "alg_bytes_per_wave_instruction": round(alg_wave) if alg_wave else None,
                         # measured bytes past L2 (FETCH_SIZE x 2 + WRITE_SIZE): fabric
                         # requests, Infinity-Cache hits included (MI355X guide, HBM
                         # section) — an upper bound of HBM traffic, not HBM itself
                         "frac_l2_miss": (round(traffic / kernel_s / 1e9 / HBM_PEAK_GBS, 4)
                                          if traffic and kernel_s > 0 else None),
                         "traffic_counts": TRAFFIC_COUNTS,
                         "kernel": ("queued pipeline (k_q_primary, k_q_segment, k_q_fallback, k_sh_*, k_q_accum; "
                                    "HIP events around the pose)" if queued else "k_paths"),
                         "alg_bytes_per_launch": round(alg_frac), "alg_bytes_parts": alg_parts,
                         "per_segment": {k: round(cs[c] / max(cs["rays"], 1), 3) for k, c in
                                         (("node_fetches", "node_fetches"), ("tri_prefilter", "tri_prefilter"),
                                          ("tri_tests_fp64", "tri_tests"), ("chain_checks", "chain_checks"))},
                         "bytes": "per-lane node steps x 96 (quantised) + wave node steps x 256 and wave triangle "
                                  "records x 48 (primary segments walked by the wave) + pre-filter x 48 + fp64 tests "
                                  "x 72 + chain checks x 52 + segments x 56 + 3 per pixel; queued: + 160 per bounce "
                                  "ray and 48 per sample (queues, final radiance); occlusion rays: binned: 140 per "
                                  "ray (record + key written, key/record pairs through the 3-pass sort, record read) + 48 per lit one + wave node steps x 256 + "
                                  "wave triangle records x 48; per lane: node steps x 96 + triangle records x 48 "
                                  "(+ 64 per record and 48 per lit one from queued records)",
                         "convention": "a record once per fetching wave instruction: the wave walks' (primary, "
                                       "occlusion) nodes and triangles once per wave, the per-lane bounce walks' "
                                       "per lane (each lane's node is its own fetch)",
                         "wave_nodes_per_pose": round(cs["wave_nodes"] / F), "wave_tris_per_pose": round(cs["wave_tris"] / F),
                         "valu": valu},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def paths_cpu_baseline(tris, a, path, W, H, S, B, shadow=True, pose=0, gpu_rgb=None):
    """The oracle's path tracer (the reference has none: kind "port") on host
    cores over whole rows of the same pose (the last timed one, frame = pose)
    until ~cpu_seconds.  gpu_rgb: that pose's timed colours [H, W, 3]; every
    row the oracle renders is compared with them (verified_timed_rows)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    host = host_cores()
    threads = int(os.environ.get("RT_CPU_THREADS", host["usable"]))
    b = pyoracle.Oracle().bvh(tris, a.algo, a.k)
    pos, d = path.circular_path(pose)
    check = {"pose": pose, "rows": 0, "row_list": [], "pixels": 0, "rgb_diff": 0}

    def leg(nthreads, budget_s, verify):
        rows, spent, j = 0, 0.0, 0
        n = max(1, nthreads // 4)  # whole rows per call, spread over the image
        while spent < budget_s and rows < H:
            m = min(n, H - j)
            t0 = time.perf_counter()
            o = b.render_paths(pos, d, W, H, pose, S, B, row0=j, nrows=m, threads=nthreads, shadow=shadow)
            spent += time.perf_counter() - t0
            if verify and gpu_rgb is not None:  # (outside the timed CPU work)
                check["rows"] += m
                check["row_list"].append([j, m])
                check["pixels"] += m * W
                check["rgb_diff"] += int(np.count_nonzero(np.any(o["rgb"] != gpu_rgb[j:j + m].reshape(-1, 3),
                                                                 axis=1)))
            rows += m
            j = (j + 97 * n) % (H - n)
        return rows, spent

    rows, spent = leg(threads, a.cpu_seconds, True)
    rows1, spent1 = leg(1, a.cpu_seconds / 3, False)
    rate = lambda r, s: round(r * W * S * (1 + B) / s / 1e6, 4)
    return {"value": rate(rows, spent), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{rows} rows of {W} px x {S} spp x (1 + {B}) segments, pose {pose} ({spent:.1f} s)",
            **({"verified_timed_rows": dict(check, equal=check["rgb_diff"] == 0 and check["rows"] > 0,
                                            compared="PPM bytes of the timed pose (the timed call writes colours "
                                                     "and the hit count only)")}
               if gpu_rgb is not None else {}),
            "all_cores": {"value": rate(rows, spent), "cores": threads},
            "one_core": {"value": rate(rows1, spent1), "cores": 1,
                         "sample": f"{rows1} rows of {W} px, pose {pose} ({spent1:.1f} s)"},
            "host": host,
            "note": "nominal rays (W x H x spp x (1 + bounces)) per second, as the GPU line; the reference has "
                    "no path tracer, so the oracle's restatement of this build's model is timed"}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import raytracingdemo_amd as rt
    from raytracingdemo_amd.scenes import armadillo_scene, sponza_scene
    from raytracingdemo_amd.shards import deinterleave_into, gather_frames, rows_per_rank, shard_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    # RT_BENCH_REHEARSE=1: rehearse the N-rank path on ONE GPU (every rank on
    # device 0, gloo over host copies instead of RCCL); numbers are not valid
    rehearse = world > 1 and os.environ.get("RT_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            # the gathers run on a high-priority RCCL stream: the persistent
            # render grid holds every CU's wave slots, and a collective's
            # workgroups should take the first ones a launch frees
            try:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
            except (AttributeError, RuntimeError):  # (a build without the option: default streams)
                opts = None
            dist.init_process_group("nccl", device_id=dev, pg_options=opts)
    coll = (lambda t: t.cpu()) if rehearse else (lambda t: t)  # collective-side tensors
    ranks = rank_facts(a, world, rank, local, dev, coll, rehearse) if world > 1 else None

    if a.scene == "armadillo":
        sc = armadillo_scene()
        if sc is None:
            raise SystemExit("config c3 needs RT_ARMADILLO_OBJ=<armadillo.obj> (stripped from the reference)")
        tris, label = sc
    else:
        tris, label = sponza_scene()
    # the scene: reference tree on the host, walk tree built on this GPU
    # (rt_scene_create_on_device), then the replica upload; the stage times
    # are the reference's dynamic-scene metric (build + traversal,
    # scripts/bvh_analysis.py:62,543) next to the host walk-tree build
    t_build = time.perf_counter()
    # (RT_BENCH_HOST_WALK=1: the walk tree built on the host, for A/B runs)
    wdev = None if os.environ.get("RT_BENCH_HOST_WALK") == "1" else local
    scene = rt.Scene(tris, a.algo, a.k, walk_device=wdev)
    t_upload = time.perf_counter()
    scene.upload([local])
    torch.cuda.synchronize(dev)
    t_ready = time.perf_counter()
    bt = scene.build_times()
    # a second build: the first one in a process also loads the build kernels
    warm_scene = rt.Scene(tris, a.algo, a.k, walk_device=wdev)
    warm = warm_scene.build_times()
    t_wu = time.perf_counter()
    warm_scene.upload([local])
    torch.cuda.synchronize(dev)
    upload_warm_ms = (time.perf_counter() - t_wu) * 1e3
    del warm_scene
    build_ms = {"scene_create_ms": round((t_upload - t_build) * 1e3, 1),
                "walk_tree_device_warm_ms": round(warm["walk_tree_ms"], 1),
                # (the reference tree and the walk tree build at the same time)
                "scene_create_warm_ms": round(warm["total_ms"], 1),
                "reference_tree_ms": round(bt["reference_tree_ms"], 1),
                "walk_tree_device_ms": round(bt["walk_tree_ms"], 1),
                "flatten_ms": round(bt["flatten_ms"], 1), "soup_ms": round(bt["soup_ms"], 1),
                "upload_ms": round((t_ready - t_upload) * 1e3, 1), "upload_warm_ms": round(upload_warm_ms, 1)}
    if world == 1 and not a.paths:
        hb = rt.Scene(tris, a.algo, a.k).build_times()
        build_ms["walk_tree_host_ms"] = round(hb["walk_tree_ms"], 1)
        build_ms["scene_create_host_walk_ms"] = round(hb["total_ms"], 1)
    if a.paths:
        return run_paths(a, scene, tris, label, world, rank, local, dev, coll, rehearse, ranks)
    st = scene.stats()
    W, H, F = a.width, a.height, a.frames
    center = rt.scene_center(tris)
    path = rt.CameraPath(center, 36)
    cams = [path.circular_path(f % 36) for f in range(F)]

    # row shard of this process: rank of world (--shard-of N at one process:
    # shard 0 of N, a diagnostic of the per-GPU work at N ranks)
    srank, sworld = (0, a.shard_of) if (world == 1 and a.shard_of > 1) else (rank, world)
    rows = rows_per_rank(H, sworld)            # rows per rank (padded)
    my_rows = len(shard_rows(srank, sworld, H))
    S = a.spp
    # Two buffer sets and two streams: step k renders into set k % 2 on
    # stream k % 2, so the library runs consecutive steps' launches
    # concurrently (step k + 1's waves fill the CUs step k's tail leaves idle;
    # include/rt.h "Device ordering"), and with N > 1 the gather of step k
    # overlaps the render of step k + 1 (the render of step k + 2 waits for
    # the gather of step k).  --no-overlap: one stream.
    NB = 2
    ids = [torch.empty((F, rows, W, S), dtype=torch.int32, device=dev) for _ in range(NB)]
    # per-sample hit distance |hit - o| (stack_bvh.hpp:631), written in the timed region
    dists = [torch.empty((F, my_rows, W, S), dtype=torch.float64, device=dev) for _ in range(NB)]
    # a step's payload per buffer set: the rgb frames, then the per-frame hit
    # counts (8-B aligned), so that a step ships with ONE collective
    rgb_bytes = F * rows * W * 3
    cnt_off = (rgb_bytes + 7) // 8 * 8
    pay_bytes = cnt_off + F * 8
    pay = [torch.zeros(pay_bytes, dtype=torch.uint8, device=dev) for _ in range(NB)]
    rgb = [p[:rgb_bytes].view(F, rows, W, 3) for p in pay]
    cnt = [p[cnt_off:].view(torch.int64) for p in pay]
    # the library writes frame f at f * W * my_rows: a short shard renders
    # into contiguous buffers and is copied into the padded gather layout
    padded = my_rows != rows
    r_ids = [torch.empty((F, my_rows, W, S), dtype=torch.int32, device=dev) for _ in range(NB)] if padded else ids
    r_rgb = [torch.zeros((F, my_rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(NB)] if padded else rgb
    # rank 0's gather buffers, allocated once: [world, F, rows, W, 3], and the
    # de-interleaved frames [F, H, W, 3] (the step's framebuffers) and counts
    root = world > 1 and rank == 0
    # diagnostic (RT_BENCH_SHIP_SIM=1 with --shard-of N at one process): rank
    # 0's side of the gather on this one GPU — the N shards' rgb copied into
    # the gather buffer on the side stream, then the de-interleave — to see
    # whether side-stream work keeps pace with the overlapped renders
    # (=1: every shard copied by rank 0's CUs; =2: only its own shard, the
    # peers' shards written over xGMI by their senders, as RCCL's P2P
    # transport does; =3: no de-interleave either)
    ship_sim = int(os.environ.get("RT_BENCH_SHIP_SIM", "0")) if world == 1 and sworld > 1 else 0
    ng = sworld if ship_sim else world
    # rank 0's gathered payloads [ng, pay_bytes], seen as rgb [ng, F, rows, W, 3]
    # and counts [ng, F]
    gather_pay = [coll(pay[0]).new_empty((ng, pay_bytes)) for _ in range(NB)] if root or ship_sim else None
    gather_rgb = [g[:, :rgb_bytes].view(ng, F, rows, W, 3) for g in gather_pay] if gather_pay else None
    gather_cnt = [g[:, cnt_off:].view(torch.int64) for g in gather_pay] if gather_pay else None
    frames = ([torch.empty((F, H, W, 3), dtype=torch.uint8, device=dev) for _ in range(NB)]
              if root or ship_sim else None)
    stream = torch.cuda.current_stream(dev)
    streams = [stream, stream if a.no_overlap else torch.cuda.Stream(dev)]  # buffer set b renders on streams[b]
    post = torch.cuda.Stream(dev, priority=-1) if world > 1 or ship_sim else None  # gather + de-interleave
    shipped = [None] * NB                                 # event: set b's gather and copy done
    # Rank 0 de-interleaves step k's gathered shards inside the render of step
    # k + 2 (the next render into the same buffer set, which waits for that
    # gather anyway): the render's traversal waves copy the rows between their
    # tiles (rt_render_shard_device_job), where a separate kernel would wait
    # for the persistent grid to drain and then hold the GPU (RT_BENCH_SHIP_SIM
    # on one GPU: -10% at the per-GPU size of 8 GPUs).  pending[b]: set b's
    # gathered shards are not de-interleaved yet; the timed region ends after
    # the last ones are.  RT_BENCH_FUSED_DEINT=0: a de-interleave kernel per step.
    fused_deint = os.environ.get("RT_BENCH_FUSED_DEINT", "1") != "0" and not rehearse
    # With an exchange (N > 1, or its simulation) every render leaves one
    # workgroup slot per CU free (RT_FLAG_SIDE_SLOT), so the gather's RCCL
    # kernels run beside the next render instead of waiting for its persistent
    # grid to drain: on one GPU at the per-GPU size of 8 GPUs, a one-rank RCCL
    # gather of the 28-MB payload finished 0.23 ms after its render instead
    # of 0.69 ms, the simulated rank-0 step took 0.612 instead of 0.670 ms,
    # and the render alone 0.565 vs 0.566 ms (tools/exchange_probe.py,
    # DESIGN.md §8).  RT_BENCH_SIDE_SLOT=0 turns it off.
    side_slot = (world > 1 or ship_sim > 0) and os.environ.get("RT_BENCH_SIDE_SLOT", "1") != "0"
    pending = [False] * NB
    mode = a.mode
    zero_fill = os.environ.get("RT_BENCH_ZERO_FILL") == "1"

    def render(b, timing=False, count=False):
        # the whole camera orbit in one batched call (the library launches up
        # to 36 frames per walk / fix-up launch)
        sb = streams[b]
        job = None
        if pending[b]:
            job = deint_job(b)
            pending[b] = False
        with torch.cuda.stream(sb):
            if shipped[b] is not None:
                sb.wait_event(shipped[b])  # set b's previous gather has read it
            # the library's multi-GPU partition (rt_render_shard_device: bands of
            # 8 rows interleaved over the ranks); the render stores the per-pose
            # hit counts (RT_FLAG_COUNTS_STORE), so no zero fill precedes it —
            # one would wait behind the other stream's persistent grid for
            # ~3 ms and gate this render's start
            if zero_fill:  # (RT_BENCH_ZERO_FILL=1: round 5's fill + adding call, for A/B runs)
                cnt[b].zero_()
            scene.render_shard_device(local, cams, W, H, srank, sworld, hit_id=r_ids[b].data_ptr(),
                                      dist=dists[b].data_ptr(), rgb=r_rgb[b].data_ptr(), hit_count=cnt[b].data_ptr(),
                                      stream=sb.cuda_stream, mode=mode, timing=timing, count=count, spp=S, job=job,
                                      side_slot=side_slot, counts_store=not zero_fill)
            if padded:
                ids[b][:, :my_rows] = r_ids[b]
                rgb[b][:, :my_rows] = r_rgb[b]

    def deint_job(b):
        # rank 0's de-interleave of set b's gathered payloads into frames[b]
        # (include/rt.h rt_deinterleave_job: block = one rank's payload)
        return dict(gathered=gather_pay[b].data_ptr(), block_bytes=pay_bytes, section_offset=0, shards=ng, frames=F,
                    height=H, width=W, elem_bytes=3, frame_rows=rows, frames_out=frames[b].data_ptr())

    def deinterleave_now(b, st):
        # the same de-interleave as its own kernel on stream st (the library's
        # job with nothing to render), or on the host copies of a rehearsal
        if gather_pay[b].is_cuda:
            scene.render_shard_device(local, [], W, H, 0, 1, stream=st.cuda_stream, job=deint_job(b))
        else:
            deinterleave_into(gather_rgb[b], H, frames[b])

    def ship(b):
        # the step's framebuffers (rgb) and per-frame hit counts
        # to rank 0 with RCCL, issued on a side stream after the render, and
        # de-interleaved there (image row j = r * world + rank) into frames[b]
        if ship_sim:
            post.wait_stream(streams[b])
            with torch.cuda.stream(post):
                for g in range(sworld if ship_sim == 1 else 1):
                    gather_pay[b][g].copy_(pay[b])
                if ship_sim != 3 and fused_deint:
                    pending[b] = True
                elif ship_sim != 3:
                    deinterleave_now(b, post)
                ev = torch.cuda.Event()
                ev.record(post)
            shipped[b] = ev
            return
        if world == 1:
            return
        post.wait_stream(streams[b])
        with torch.cuda.stream(post):
            # (rehearsal: the same call on host copies over gloo)
            w = dist.gather(coll(pay[b]), list(gather_pay[b].unbind(0)) if root else None, dst=0, async_op=True)
            w.wait()
            if root and fused_deint:
                pending[b] = True  # de-interleaved by the render of step k + 2 (or drain())
            elif root:
                deinterleave_now(b, post)
            ev = torch.cuda.Event()
            ev.record(post)
        shipped[b] = ev

    def render_step(k, timing=False, count=False):
        b = k % NB
        render(b, timing=timing, count=count)
        ship(b)

    def drain():
        if post is not None:
            with torch.cuda.stream(post):
                for b in range(NB):
                    if pending[b]:
                        deinterleave_now(b, post)
                        pending[b] = False
            stream.wait_stream(post)

    # counting pass for algorithmic bytes (outside the timed region)
    render(0, count=True)
    torch.cuda.synchronize(dev)
    cs = scene.frame_stats(local, reset=True)
    nb = st["node_bytes"]
    # SURVEY.md 8(d)'s per-ray figure: what each ray's own traversal touches
    survey_bytes_per_ray = (cs["node_fetches"] * nb + cs["tri_prefilter"] * TRI32_BYTES + cs["tri_tests"] * TRI64_BYTES +
                            cs["rays"] * OUT_BYTES) / max(cs["rays"], 1)
    fused = cs["wave_tiles"] and os.environ.get("RT_RESOLVE", "")[:1] != "s"
    walk_bytes = cs["wave_nodes"] * nb + cs["wave_tris"] * TRI32_BYTES
    conventions = None
    if fused:
        # packet traversal kernel with the fused resolve (the dominant kernel),
        # every record counted once per wave: a node or fp32 triangle record
        # fetched once for the wave's 64 rays, and the fp64 records the lanes
        # resolve counted once per wave-distinct triangle (the Moller-Trumbore
        # part per candidate, the shading part per winner: neighbouring rays
        # test and hit the same triangles); per lane the ancestor boxes
        # re-verified and the outputs (rays are generated in-kernel: no camera
        # reads; spp > 1: per sample its outputs, colour and status)
        out_bytes = cs["rays"] * (OUT_BYTES if S == 1 else
                                  PACKED_SAMPLE_BYTES + 3.0 / S if packed_spp(S) else SAMPLE_BYTES)
        resolve_lane = cs["tri_tests"] * MT64_BYTES + cs["hits"] * WIN_BYTES + cs["chain_nodes"] * CHAIN_BYTES
        resolve_wave = (cs["wave_tri_tests"] * MT64_BYTES + cs["wave_winners"] * WIN_BYTES +
                        cs["chain_nodes"] * CHAIN_BYTES)
        trace_bytes = walk_bytes + resolve_wave + out_bytes
        conventions = {"per_wave": trace_bytes / F, "walk_only": walk_bytes / F,
                       "walk_and_outputs": (walk_bytes + out_bytes) / F,
                       "per_lane_resolve": (walk_bytes + resolve_lane + out_bytes) / F}
    elif cs["wave_tiles"]:
        # packet traversal kernel, split resolve: the walk plus the candidate
        # lists it writes
        trace_bytes = (cs["wave_nodes"] * nb + cs["wave_tris"] * TRI32_BYTES +
                       cs["rays"] * 1 + cs["tri_tests"] * CAND_BYTES)
    else:  # per-lane kernel: each ray fetches its own records
        trace_bytes = (cs["node_fetches"] * nb + cs["tri_prefilter"] * TRI32_BYTES + cs["tri_tests"] * TRI64_BYTES +
                       cs["chain_nodes"] * CHAIN_BYTES + cs["rays"] * OUT_BYTES)
    alg_bytes_per_frame = trace_bytes / F
    # warm-up with kernel timing on, so the library's per-launch timing events
    # exist before the timed region (they are recycled, not re-created): W
    # steps, then render-only steps (no gather, so ranks may run different
    # counts) until at least SETTLE_S of continuous GPU work has passed — the
    # MI355X raises its clock over the first ~25 ms of load (tools/step_trace.py:
    # 5.58 -> 4.55 ms per step over the first 5 steps), and the timed steps
    # follow the settle with no idle gap but the barrier
    ktiming = not os.environ.get("RT_BENCH_NO_KTIMING")
    settled = 0
    for k in range(a.warmup):
        render_step(k, timing=ktiming)
    drain()
    t_set = time.perf_counter()
    while time.perf_counter() - t_set < SETTLE_S:
        render(settled % NB, timing=ktiming)
        torch.cuda.synchronize(dev)
        settled += 1
    scene.frame_stats(local, reset=True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        render_step(k, timing=ktiming)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # multi-rank (outside the timed region): the last step's gathered,
    # de-interleaved frames and hit counts, and a gather of the last step's
    # hit ids, must equal a full-image render on rank 0
    verified = None
    if world > 1:
        bl = (a.steps - 1) % NB
        g_ids = gather_frames(coll(ids[bl]), H, world, rank)
        torch.cuda.synchronize(dev)
        if rank == 0:
            f_ids = torch.empty((F, H, W, S), dtype=torch.int32, device=dev)
            f_rgb = torch.empty((F, H, W, 3), dtype=torch.uint8, device=dev)
            f_cnt = torch.zeros((F,), dtype=torch.int64, device=dev)
            scene.render_batch_device(local, cams, W, H, 0, 1, H, hit_id=f_ids.data_ptr(), rgb=f_rgb.data_ptr(),
                                      hit_count=f_cnt.data_ptr(), stream=stream.cuda_stream, mode=mode, spp=S)
            torch.cuda.synchronize(dev)
            verified = bool(torch.equal(g_ids.to(dev), f_ids) and torch.equal(frames[bl], f_rgb) and
                            torch.equal(gather_cnt[bl].to(dev).sum(0), f_cnt))
        dist.barrier()
    # per-kernel HIP-event times of the timed launches (library stream)
    ks = scene.frame_stats(local, reset=True)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        t = coll(t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_rays = a.steps * F * W * (H if sworld == world else my_rows) * S
    value = total_rays / elapsed / 1e6
    launches_timed = max(ks["timed_launches"], 1)
    frames_timed = a.steps * F
    frame_s = elapsed / frames_timed
    # dominant (traversal) kernel, HIP events around each of its launches
    # (one launch = up to 36 frames); without library timing, whole frames
    trace_s = ks["trace_ms"] * 1e-3 if ks["timed_launches"] else elapsed
    avg_kernel_s = trace_s / launches_timed if ks["timed_launches"] else frame_s
    # With consecutive launches on two streams the HIP-event span of a launch
    # also covers the wait for the previous launch's waves to drain (its
    # start event fires when its stream reaches it), so spans overlap and
    # their mean exceeds the time each launch actually holds the GPU.  The
    # roofline then takes the wall time per launch of the timed region
    # (launches back to back, gaps included: an upper bound; in a rocprofv3
    # kernel trace it is the union of the timed launches' busy intervals per
    # launch, `tools/launch_ends.py`, not their own start-to-end durations,
    # which overlap) and reports the mean span beside it.
    span_s = avg_kernel_s
    overlapped = not a.no_overlap and ks["timed_launches"] > 1
    if overlapped:
        avg_kernel_s = min(avg_kernel_s, elapsed / launches_timed)
    frames_per_launch = frames_timed / launches_timed if ks["timed_launches"] else 1.0
    alg_bytes_per_launch = alg_bytes_per_frame * frames_per_launch
    achieved = alg_bytes_per_launch / avg_kernel_s / 1e9
    # the same kernel time against the other byte conventions (GB/s)
    rates = ({k: v * frames_per_launch / avg_kernel_s / 1e9 for k, v in conventions.items()}
             if conventions else {})

    if rank == 0:
        key = (f"{label}|{W}x{H}|{a.algo}-{a.k}|{mode}|n{world}|fpl{frames_per_launch:g}" + (f"|spp{S}" if S > 1 else "")
               + ("|fused" if fused else "") + (f"|shard-of{sworld}" if sworld != world else ""))
        if a.key_out:
            with open(a.key_out, "w") as fh:
                fh.write(key + "\n")
        traffic = None
        try:
            pm = json.load(open(a.pmc))
            if pm.get("workload_key") == key:
                traffic = round(float(pm["hbm_bytes_per_launch"]))
        except (OSError, ValueError, KeyError):
            pass
        # VALU issue utilisation of the same kernel (committed SQ PMC passes,
        # tools/pmc_valu.py): the walk is issue-bound, not HBM-bound
        valu = None
        try:
            pv = json.load(open(os.path.join(ROOT, "profiles", "pmc_valu.json")))
            if pv.get("workload_key") == key:
                valu = {"busy": pv["valu_busy"], "issue": issue_roofline(pv), "insts_per_launch": pv["valu_insts_per_launch"],
                        "salu_insts_per_launch": pv["salu_insts_per_launch"],
                        # SURVEY §8(d) asks for VALU ops per ray: every lane of a
                        # wave64 instruction is one ray's op (a tile's 64 rays share
                        # the wave's node and triangle tests)
                        "lane_ops_per_ray": round(64 * pv["valu_insts_per_launch"] / (frames_per_launch * W * H * S), 1),
                        "wave_cycles_split": pv["wave_cycles_split"], "source": "profiles/pmc_valu.json"}
        except (OSError, ValueError, KeyError):
            pass
        cpu = None
        dropin = None
        if world == 1 and not a.no_dropin and S == 1:
            dropin = dropin_rate(scene, cams, W, H, mode)
            dropin["fused_shade"] = dropin_rate(scene, cams, W, H, mode, want=("rgb",))
        if world == 1 and not a.no_cpu:
            # the timed step's frames (buffer set 0, the last step at N = 1)
            # checked against the reference frames the baseline renders
            gpu = None
            if S == 1 and sworld == 1 and F <= 36:
                gpu = {"ids": ids[0][:, :H, :, 0].reshape(F, H * W).cpu().numpy(),
                       "dist": dists[0][:, :H, :, 0].reshape(F, H * W).cpu().numpy(),
                       "rgb": rgb[0][:, :H].reshape(F, H * W, 3).cpu().numpy(), "cnt": cnt[0].cpu().numpy()}
            cpu = cpu_baseline(tris, a.algo, a.k, cams, W, H, a.cpu_seconds, gpu=gpu)
        line = {
            "metric": METRIC if S == 1 else METRIC.replace("1spp", f"{S}spp"), "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "settle_steps": settled,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32 traversal + f64 exact resolve",
            "data": f"synthetic: {label}",
            "config": {"workload": f"{label}, {W}x{H}x{S}spp primary rays, {a.algo}-{a.k} (BVH{a.k}) k-way, "
                                   f"{F}-frame camera orbit per step",
                       "width": W, "height": H, "spp": S, "bvh": f"{a.algo}-{a.k}", "frames_per_step": F,
                       "triangles": int(st["triangles"]), "mode": mode,
                       **({"diagnostic_shard_of": sworld} if sworld != world else {}),
                       **({"diagnostic_ship_sim": ship_sim} if ship_sim else {}),
                       **({"side_slot": True} if side_slot else {}),
                       "parallelism": f"8-row image bands interleaved x{world}" +
                                      (" + RCCL gather of rgb (overlapped)" if world > 1 else ""),
                       **({"gather_verified": verified,
                           # what the timed gather ships (SURVEY 8(e) names hit id + dist + rgb)
                           "timed_gather_payload": "rgb frames + per-pose hit counts (RCCL gather to rank 0 and "
                                                   "de-interleave, overlapped with the next render); hit ids and "
                                                   "distances stay on the ranks in the timed region and are gathered "
                                                   "after it, for gather_verified (DESIGN.md §8)"}
                          if world > 1 else {}),
                       # rank 0's de-interleave of the gathered frames: done by the
                       # traversal kernel of a render (rt_render_shard_device_job) or
                       # by its own kernel, over the timed steps
                       **({"side_jobs": {"fused": ks["side_jobs_fused"], "kernel": ks["side_jobs_kernel"]}}
                          if ks["side_jobs_fused"] + ks["side_jobs_kernel"] else {}),
                       **({"ranks": {**ranks, "gather_bytes_per_step": world * pay_bytes}} if ranks else {}),
                       **({"rehearsal_not_a_measurement": True} if rehearse else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         **({"convention": "every record once per wave (walk nodes and fp32 triangles per node "
                                           "step; fp64 records per wave-distinct triangle tested / won); ancestor "
                                           "boxes and outputs per ray",
                             "frac_walk": round(rates["walk_only"] / HBM_PEAK_GBS, 4),
                             "frac_walk_and_outputs": round(rates["walk_and_outputs"] / HBM_PEAK_GBS, 4),
                             "frac_per_lane_resolve": round(rates["per_lane_resolve"] / HBM_PEAK_GBS, 4),
                             **({"frac_l2_miss": round(traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                                 "traffic_counts": TRAFFIC_COUNTS}
                                if traffic else {})} if rates else {}),
                         "valu": valu,
                         "kernel": ("k_trace_packet (walk + fused exact resolve)" if fused else
                                    "k_trace_packet (walk)" if cs["wave_tiles"] else "k_trace_exact"),
                         "kernel_ms_avg": round(avg_kernel_s * 1e3, 4),
                         "kernel_time_basis": ("wall time per launch (launches overlapped on two streams)"
                                               if overlapped and avg_kernel_s < span_s else
                                               "HIP events around each launch on its stream"),
                         "kernel_ms_span_avg": round(span_s * 1e3, 4),
                         "alg_bytes_per_launch": int(alg_bytes_per_launch),
                         "frames_per_launch": round(frames_per_launch, 3),
                         "alg_bytes_per_frame": int(alg_bytes_per_frame),
                         "trace_ms_per_frame": round(trace_s / frames_timed * 1e3, 4),
                         "frame_ms_avg": round(frame_s * 1e3, 4),
                         "survey_bytes_per_ray": round(survey_bytes_per_ray, 1),
                         "per_ray": {"node_fetches": round(cs["node_fetches"] / max(cs["rays"], 1), 3),
                                     "tri_prefilter": round(cs["tri_prefilter"] / max(cs["rays"], 1), 3),
                                     "tri_tests_fp64": round(cs["tri_tests"] / max(cs["rays"], 1), 3),
                                     "wave_tri_tests_per_tile": round(cs["wave_tri_tests"] / max(cs["wave_tiles"], 1), 2),
                                     "wave_winners_per_tile": round(cs["wave_winners"] / max(cs["wave_tiles"], 1), 2),
                                     "chain_checks": round(cs["chain_checks"] / max(cs["rays"], 1), 4),
                                     "chain_nodes": round(cs["chain_nodes"] / max(cs["rays"], 1), 4),
                                     "wave_nodes_per_tile": round(cs["wave_nodes"] / max(cs["wave_tiles"], 1), 2),
                                     "wave_leaves_per_tile": round(cs["wave_leaves"] / max(cs["wave_tiles"], 1), 2),
                                     "wave_tris_per_tile": round(cs["wave_tris"] / max(cs["wave_tiles"], 1), 2),
                                     "redo_rays": round(cs["redo_rays"] / max(cs["rays"], 1), 7),
                                     "redo_chain": round(cs["redo_chain"] / max(cs["rays"], 1), 7),
                                     "spilled_rays": round(cs["spilled_rays"] / max(cs["rays"], 1), 7),
                                     "dropped_rays": round(cs["dropped_rays"] / max(cs["rays"], 1), 7),
                                     "node_bytes": st["node_bytes"], "tri32_bytes": TRI32_BYTES,
                                     "tri64_bytes": TRI64_BYTES}},
            "cpu_baseline": cpu,
            "dropin_frame_path": dropin,
            "scene_build": build_ms,
            "scene_difficulty": scene_difficulty(label, a.algo, a.k),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def issue_roofline(pv):
    """The instruction-issue bound beside the HBM one (the walk is cache-resident
    and issue/latency-bound): the share of the SIMDs' issue
    cycles the kernel's VALU (2 cycles per wave64 instruction on a SIMD-32)
    and SALU (1 cycle) instructions take, from the committed SQ passes
    (tools/pmc_valu.py): (2 VALU + SALU) / (1024 SIMDs x active cycles)."""
    cyc = pv.get("cycles_per_xcd")
    valu, salu = pv.get("valu_insts_per_launch"), pv.get("salu_insts_per_launch")
    if not (cyc and valu and salu):
        return None
    return {"frac": round((2.0 * valu + salu) / (1024.0 * cyc), 4), "valu": round(2.0 * valu / (1024.0 * cyc), 4),
            "salu": round(salu / (1024.0 * cyc), 4), "unit": "issue cycles / SIMD cycles",
            "formula": "(2 x SQ_INSTS_VALU + SQ_INSTS_SALU) / (1024 x GRBM_GUI_ACTIVE / 8)",
            # the two ports apart: VALU per SIMD, SALU on the CU's one scalar unit
            "valu_port": round(2.0 * valu / (1024.0 * cyc), 4), "salu_port_per_cu": round(salu / (256.0 * cyc), 4)}


def packed_spp(spp):
    """The library's fp.pack rule (rt_api.cpp frame_params): with the fused
    resolve, spp 4 and 16 put all samples of a pixel in one wave (its colours
    summed across lanes, no k_average)."""
    return (spp > 1 and 64 % spp == 0 and os.environ.get("RT_SPP_PACK", "1")[:1] != "0"
            and os.environ.get("RT_RESOLVE", "")[:1] != "s")


def dropin_rate(scene, cams, W, H, mode, want=("hit_id", "pos")):
    """The drop-in path INTEGRATION.md §2 binds (rt_render_frame: one pose per
    call into host buffers, blocking, as runTest's calculateScreen call,
    src/main.cpp:253-255) for every pose of the orbit, D2H copies included.
    want: the outputs copied back — ("hit_id", "pos") is what
    gpu_calculate_screen requests (28 B per pixel: runTest rebuilds ray_hits
    from them and shades on the host); ("rgb",) is the fused-shadeScreen
    variant of §2 (the PPM bytes and the hit count, 3 B per pixel).
    Reported beside the headline, never as it."""
    # one set of host arrays reused frame after frame, as runTest reuses its
    # global ray_hits (src/main.cpp:39)
    g = None
    for p, d in cams[:2]:
        g = scene.calculate_screen(p, d, W, H, mode=mode, want=want, out=g)
    t0 = time.perf_counter()
    dev_s = 0.0
    for p, d in cams:
        g = scene.calculate_screen(p, d, W, H, mode=mode, want=want, out=g)
        dev_s += g["seconds"]
    wall = time.perf_counter() - t0
    n = len(cams) * W * H
    return {"value": round(n / wall / 1e6, 2), "unit": "Mrays/s", "entry_point": "rt_render_frame",
            "outputs": list(want), "frames": len(cams), "ms_per_frame": round(wall / len(cams) * 1e3, 3),
            "device_ms_per_frame": round(dev_s / len(cams) * 1e3, 3),
            "note": "one pose per call into one reused set of pageable host arrays, blocking"}


if __name__ == "__main__":
    main()
