"""GPU parity at the benchmarked sizes: the exact workload bench.py times
(sponza proxy, 1920x1080, bsah-8, the 36-pose orbit of runTest in one
rt_render_batch_device call, 36 poses per launch) against the oracle on full
frames, pixel for pixel; config c4 (4 spp) on full frames; config c3
(armadillo) where its geometry is supplied; and the candidate-overflow pool
running dry.  Reference: StackBVH::traverse (src/stack_bvh.hpp:611-644),
runTest's pose loop (src/main.cpp:234-281), shadeScreen (src/main.cpp:351-381).
"""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from conftest import golden_scene

pytestmark = pytest.mark.gpu

rt = pytest.importorskip("raytracingdemo_amd")
torch = pytest.importorskip("torch")

W, H = 1920, 1080
_PROXY: dict = {}


def proxy():
    if "s" not in _PROXY:
        from raytracingdemo_amd.scenes import sponza_proxy_triangles
        tris = sponza_proxy_triangles()
        _PROXY["tris"] = tris
        _PROXY["s"] = rt.Scene(tris, "bsah", 8).upload([0])
    return _PROXY["tris"], _PROXY["s"]


def orbit(tris, n=36):
    path = rt.CameraPath(rt.scene_center(tris), 36)
    return [path.circular_path(f) for f in range(n)]


def render_orbit(s, cams, spp=1, count=False):
    """bench.py's call: every pose of `cams`, full frames, device buffers."""
    F = len(cams)
    ids = torch.empty((F, H, W, spp), dtype=torch.int32, device="cuda:0")
    dist = torch.empty((F, H, W, spp), dtype=torch.float64, device="cuda:0")
    rgb = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
    cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ids.data_ptr(), dist=dist.data_ptr(), rgb=rgb.data_ptr(),
                          hit_count=cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream, spp=spp,
                          count=count)
    torch.cuda.synchronize()
    return ids, dist, rgb, cnt


@pytest.mark.parametrize("rays", ["1", "2"])
def test_headline_orbit_full_size_matches_oracle(oracle, monkeypatch, rays):
    """All 36 poses at 1920x1080 through the fused pipeline (as timed; rays
    per lane of the packet kernel: 1 — 8x8 tiles, 2 — 16x8 tiles,
    k_trace_packet_r), then the split resolve (k_resolve, the spp > 1 path) on
    the same call: hit ids, distances, PPM bytes and per-frame hit counts equal
    the oracle's full frames; the counting pass reports every ray and no lost
    pixel."""
    monkeypatch.setenv("RT_PACKET_RAYS", rays)
    tris, s = proxy()
    cams = orbit(tris)
    ids, dist, rgb, cnt = render_orbit(s, cams)
    ob = oracle.bvh(tris, "bsah", 8)
    hits_total = 0
    for f, (p, d) in enumerate(cams):
        o = ob.render(p, d, W, H, want=("id", "dist", "rgb"))
        g_id = ids[f].cpu().numpy().reshape(-1).view(np.uint32)
        gid = np.where(g_id == rt.RT_MISS, -1, g_id.astype(np.int64))
        assert np.array_equal(gid, o["id"]), (f, np.flatnonzero(gid != o["id"])[:8])
        m = o["id"] >= 0
        gd = dist[f].cpu().numpy().reshape(-1)
        assert np.array_equal(gd[m], o["dist"][m]), f
        assert np.all(gd[~m] == -1.0), f
        assert np.array_equal(rgb[f].cpu().numpy().reshape(-1, 3), o["rgb"]), f
        assert int(cnt[f]) == o["hits"], f
        hits_total += o["hits"]
    # the split resolve (candidate lists in HBM, k_resolve) gives the same bytes
    monkeypatch.setenv("RT_RESOLVE", "split")
    ids2, dist2, rgb2, cnt2 = render_orbit(s, cams)
    assert torch.equal(ids, ids2) and torch.equal(dist, dist2) and torch.equal(rgb, rgb2) and torch.equal(cnt, cnt2)
    monkeypatch.delenv("RT_RESOLVE")
    # counting pass of the timed call: every ray once, hits agree, nothing lost
    s.frame_stats(0, reset=True)
    render_orbit(s, cams, count=True)
    fs = s.frame_stats(0, reset=True)
    assert fs["rays"] == 36 * W * H
    assert fs["hits"] == hits_total
    assert fs["wave_tiles"] == 36 * (W // (8 * int(rays))) * (H // 8)
    if rays == "1":  # (the 2-ray kernel has no overflow pool: it drops with a certified bound)
        assert fs["dropped_rays"] <= fs["spilled_rays"]
    print(f"\nheadline orbit counters: spilled {fs['spilled_rays']} dropped {fs['dropped_rays']} "
          f"redo {fs['redo_rays']} (chain {fs['redo_chain']}) of {fs['rays']} rays")


@pytest.mark.parametrize("shard_of,side_slot", [(1, False), (8, False), (8, True)])
def test_consecutive_launches_on_two_streams_equal_one_stream(shard_of, side_slot):
    """bench.py's overlapped steps: consecutive orbit renders issued on two
    streams (the library alternates its two launch slots, so launch k + 1
    runs while launch k drains) into two buffer sets, hit counts stored by
    the render (RT_FLAG_COUNTS_STORE: no zero fill between launches, stale
    counts overwritten); every set equals the one-stream render bit
    for bit (hit ids, distances, PPM bytes, per-pose hit counts), also at the
    per-GPU size of an 8-GPU run (shard 0 of 8), and with RT_FLAG_SIDE_SLOT
    (the smaller persistent grid of a multi-GPU rank) with a copy kernel on a
    third stream beside each render, as bench.py's gather."""
    tris, s = proxy()
    cams = orbit(tris)
    R = rt.shard_height(H, shard_of, 0) if shard_of > 1 else H
    F = len(cams)

    def bufs():
        return (torch.empty((F, R, W), dtype=torch.int32, device="cuda:0"),
                torch.empty((F, R, W), dtype=torch.float64, device="cuda:0"),
                torch.empty((F, R, W, 3), dtype=torch.uint8, device="cuda:0"),
                torch.full((F,), 987654321, dtype=torch.int64, device="cuda:0"))

    def render(b, st, side=False, store=True):
        with torch.cuda.stream(st):
            s.render_shard_device(0, cams, W, H, 0, shard_of, hit_id=b[0].data_ptr(), dist=b[1].data_ptr(),
                                  rgb=b[2].data_ptr(), hit_count=b[3].data_ptr(), stream=st.cuda_stream,
                                  side_slot=side, counts_store=store)

    ref = bufs()
    ref[3].zero_()
    render(ref, torch.cuda.current_stream(), store=False)  # (the adding call on zeroed counters)
    torch.cuda.synchronize()
    sets = [bufs(), bufs()]
    copies = [torch.empty_like(sets[0][2]) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    post = torch.cuda.Stream(priority=-1)
    for k in range(6):
        b = k % 2
        streams[b].wait_stream(post)  # the copy of this set's previous frames is done
        render(sets[b], streams[b], side_slot)
        if side_slot:
            post.wait_stream(streams[b])
            with torch.cuda.stream(post):
                copies[b].copy_(sets[b][2])
    torch.cuda.synchronize()
    for b in sets:
        for x, y in zip(b, ref):
            assert torch.equal(x, y)
    if side_slot:
        for c in copies:
            assert torch.equal(c, ref[2])
    assert int(ref[3].sum()) > 0


@pytest.mark.parametrize("env,spp,mode", [({}, 1, "exact"), ({}, 4, "exact"), ({"RT_SPP_PACK": "0"}, 4, "exact"),
                                          ({"RT_RESOLVE": "split"}, 1, "exact"), ({"RT_PACKET_RAYS": "2"}, 1, "exact"),
                                          ({"RT_REDO_CAP": "1", "RT_POOL_CHUNKS": "1"}, 1, "exact"),
                                          ({}, 1, "fp64")])
def test_counts_store_every_pipeline(oracle, monkeypatch, env, spp, mode):
    """RT_FLAG_COUNTS_STORE on counters holding stale values: the fused packet
    kernel's last wave stores the per-pose counts (spp 1, packed spp 4); every
    other pipeline (sample-frame tiles + k_average, the split resolve, the
    2-ray kernel, k_fixup after a redo-list overflow, the literal fp64
    kernel) has the library zero them first.  Counts equal the
    oracle's; a second call on the same counters does not add up."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tris = _dup_stack(40) if "RT_REDO_CAP" in env else golden_scene("teapot.obj")
    algo = "sah" if "RT_REDO_CAP" in env else "bsah"
    s = rt.Scene(tris, algo, 8).upload([0])
    ob = oracle.bvh(tris, algo, 8)
    if "RT_REDO_CAP" in env:
        cams = [([0.0, 0.0, 3.0], [0.0, 0.0, -1.0]), ([0.3, 0.2, 2.5], [-0.1, -0.05, -1.0])]
    else:
        cams = orbit(tris, 4)
    Wd, Hd = 160, 120
    cnt = torch.full((len(cams),), 424242, dtype=torch.int64, device="cuda:0")
    rgb = torch.empty((len(cams), Hd, Wd, 3), dtype=torch.uint8, device="cuda:0")
    for _ in range(2):
        s.render_batch_device(0, cams, Wd, Hd, 0, 1, Hd, rgb=rgb.data_ptr(), hit_count=cnt.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream, spp=spp, mode=mode, counts_store=True)
        torch.cuda.synchronize()
        for f, (p, d) in enumerate(cams):
            o = ob.render(p, d, Wd, Hd) if spp == 1 else ob.render_spp(p, d, Wd, Hd, spp)
            assert int(cnt[f]) == o["hits"] > 0, (f, int(cnt[f]), o["hits"])
            assert np.array_equal(rgb[f].cpu().numpy().reshape(-1, 3), o["rgb"]), f


@pytest.mark.parametrize("env", [{}, {"RT_PACKET_RAYS": "2"}, {"RT_RESOLVE": "split"}])
def test_render_with_side_deinterleave_job(monkeypatch, env):
    """rt_render_shard_device_job: the shard render's traversal waves also
    de-interleave a gathered buffer into full frames (bench.py's rank 0).
    Random bytes laid out as 8 padded shards of [F][rows][W][3] (frame_rows =
    rows) and as the library's compact group layout (frame_rows = 0) must come
    out as shards.deinterleave's frames, while the render itself still equals
    the plain call; with RT_PACKET_RAYS=2 the job runs as its own kernel."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from raytracingdemo_amd.shards import deinterleave, rows_per_rank
    tris, s = proxy()
    cams = orbit(tris, 6)
    F, G = len(cams), 8
    R = rt.shard_height(H, G, 3)
    rows = rows_per_rank(H, G)
    g = torch.randint(0, 256, (G, F, rows, W, 3), dtype=torch.uint8, device="cuda:0")
    want = deinterleave(g, H)
    # the library's group layout: shard k holds rt_shard_height rows per frame
    blocks = [g[k, :, :rt.shard_height(H, G, k)].contiguous().reshape(-1) for k in range(G)]
    blk = max(b.numel() for b in blocks)
    compact = torch.zeros((G, blk), dtype=torch.uint8, device="cuda:0")
    for k in range(G):
        compact[k, :blocks[k].numel()] = blocks[k]
    ref_ids = torch.empty((F, R, W), dtype=torch.int32, device="cuda:0")
    st = torch.cuda.current_stream()
    s.render_shard_device(0, cams, W, H, 3, G, hit_id=ref_ids.data_ptr(), stream=st.cuda_stream)
    for gathered, block, frows in ((g, F * rows * W * 3, rows), (compact, blk, 0)):
        out = torch.zeros((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
        ids = torch.empty((F, R, W), dtype=torch.int32, device="cuda:0")
        job = dict(gathered=gathered.data_ptr(), block_bytes=block, section_offset=0, shards=G, frames=F, height=H,
                   width=W, elem_bytes=3, frame_rows=frows, frames_out=out.data_ptr())
        s.render_shard_device(0, cams, W, H, 3, G, hit_id=ids.data_ptr(), stream=st.cuda_stream, job=job)
        torch.cuda.synchronize()
        assert torch.equal(out, want), frows
        assert torch.equal(ids, ref_ids), frows
    # nothing to render: the job alone
    out = torch.zeros((F, H, W, 3), dtype=torch.uint8, device="cuda:0")
    job["gathered"], job["block_bytes"], job["frame_rows"], job["frames_out"] = g.data_ptr(), F * rows * W * 3, rows, out.data_ptr()
    s.render_shard_device(0, [], W, H, 3, G, stream=st.cuda_stream, job=job)
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_config_c4_spp4_full_frames_match_oracle(oracle):
    """Config c4 (2x2 stratified samples) on full 1080p frames of 6 poses (one
    launch of 24 sample frames: each sample resolved in the walk kernel,
    k_average forming the pixels): per-sample ids and distances, averaged
    colours, per-pose sample hit counts."""
    tris, s = proxy()
    cams = orbit(tris)[::6]
    ids, dist, rgb, cnt = render_orbit(s, cams, spp=4)
    ob = oracle.bvh(tris, "bsah", 8)
    for f, (p, d) in enumerate(cams):
        o = ob.render_spp(p, d, W, H, 4)
        g_id = ids[f].cpu().numpy().reshape(-1, 4).view(np.uint32)
        gid = np.where(g_id == rt.RT_MISS, -1, g_id.astype(np.int64))
        assert np.array_equal(gid, o["id"]), f
        m = o["id"] >= 0
        assert np.array_equal(dist[f].cpu().numpy().reshape(-1, 4)[m], o["dist"][m]), f
        assert np.array_equal(rgb[f].cpu().numpy().reshape(-1, 3), o["rgb"]), f
        assert int(cnt[f]) == o["hits"], f


def _dup_stack(n: int) -> np.ndarray:
    """n exact copies of one triangle: every pixel that sees it has n certain
    candidates at the same distance (the reference keeps the first it visits)."""
    tri = np.array([[-1.0, -1.0, 0.0, 1.0, -1.0, 0.0, 0.0, 1.0, 0.0]])
    return np.repeat(tri, n, axis=0)


@pytest.mark.parametrize("chunks", [None, "1"])
def test_overflow_pool_and_dry_pool(oracle, monkeypatch, chunks):
    """40 coincident triangles: each covered pixel lists 8 candidates in LDS,
    24 in its pool chunk and drops the rest (certified or redone).  With a
    one-chunk pool (RT_POOL_CHUNKS=1) all lanes but one find the pool dry and
    must drop from the first overflow on.  Both equal the reference traversal."""
    if chunks:
        monkeypatch.setenv("RT_POOL_CHUNKS", chunks)
    tris = _dup_stack(40)
    # (bsah cannot split coincident centroids: the reference throws "invalid
    # split position"; sah-8 builds, and its visit order picks the winner)
    s = rt.Scene(tris, "sah", 8).upload([0])
    for mode in ("exact", "fp64"):
        g = s.calculate_screen([0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 96, 72, mode=mode)
        o = oracle.bvh(tris, "sah", 8).render([0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 96, 72)
        gid = np.where(g["hit_id"] == rt.RT_MISS, -1, g["hit_id"].astype(np.int64))
        assert np.array_equal(gid, o["id"]), mode
        assert np.array_equal(g["rgb"], o["rgb"]) and g["hits"] == o["hits"] > 0, mode
    ids = torch.empty(96 * 72, dtype=torch.int32, device="cuda:0")
    s.frame_stats(0, reset=True)
    s.render_rows_device(0, [0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 96, 72, 0, 1, 72, hit_id=ids.data_ptr(),
                         stream=torch.cuda.current_stream().cuda_stream, count=True)
    torch.cuda.synchronize()
    fs = s.frame_stats(0, reset=True)
    assert fs["spilled_rays"] > 0
    assert fs["dropped_rays"] > 0
    if chunks:
        assert fs["spilled_rays"] == 1  # the one chunk; every other lane dropped straight away
    # the same frame from two streams at once: the two launch slots each have
    # their own pool, redo list and work queue
    outs = [torch.empty(96 * 72, dtype=torch.int32, device="cuda:0") for _ in range(2)]
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    for k in range(4):
        s.render_rows_device(0, [0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 96, 72, 0, 1, 72, hit_id=outs[k % 2].data_ptr(),
                             stream=sts[k % 2].cuda_stream)
    torch.cuda.synchronize()
    for o2 in outs:
        assert torch.equal(o2, ids)
    # 4 spp through the fused resolve: samples that overflow or cannot be
    # certified send their whole pixel to k_fixup via k_average
    sp = torch.empty(96 * 72 * 4, dtype=torch.int32, device="cuda:0")
    rgb = torch.empty(96 * 72 * 3, dtype=torch.uint8, device="cuda:0")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    cam = [([0.0, 0.0, 3.0], [0.0, 0.0, -1.0])]
    s.render_batch_device(0, cam, 96, 72, 0, 1, 72, hit_id=sp.data_ptr(), rgb=rgb.data_ptr(),
                          hit_count=cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream, spp=4)
    torch.cuda.synchronize()
    o = oracle.bvh(tris, "sah", 8).render_spp([0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 96, 72, 4)
    g4 = sp.cpu().numpy().view(np.uint32).reshape(-1, 4)
    assert np.array_equal(np.where(g4 == rt.RT_MISS, -1, g4.astype(np.int64)), o["id"])
    assert np.array_equal(rgb.cpu().numpy().reshape(-1, 3), o["rgb"])
    assert int(cnt[0]) == o["hits"] > 0


@pytest.mark.parametrize("env", [{}, {"RT_SPP_PACK": "0"}, {"RT_RESOLVE": "split"}, {"RT_PACKET_RAYS": "2"}])
def test_redo_pool_overflow_retries_the_launch(oracle, monkeypatch, env):
    """The redo list is a fixed pool of entries (4 MiB), not one u32 per pose
    pixel.  RT_REDO_CAP=1 with a one-chunk candidate pool (RT_POOL_CHUNKS=1):
    the 40 coincident triangles send many pixels to the fix-up, the count
    passes the pool, and k_fixup retries the whole launch through the exact
    per-lane path, discarding the walk kernel's hit partials.  Two poses in one
    launch at 1 and 4 spp (packed tiles, sample-frame tiles + k_average, the
    split resolve) equal the oracle; hit counts are not counted twice."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("RT_POOL_CHUNKS", "1")
    tris = _dup_stack(40)
    s = rt.Scene(tris, "sah", 8).upload([0])
    ob = oracle.bvh(tris, "sah", 8)
    cams = [([0.0, 0.0, 3.0], [0.0, 0.0, -1.0]), ([0.3, 0.2, 2.5], [-0.1, -0.05, -1.0])]
    Wd, Hd = 96, 72
    st = torch.cuda.current_stream().cuda_stream
    for spp in (1, 4):
        res = {}
        for cap in (None, "1"):
            if cap:
                monkeypatch.setenv("RT_REDO_CAP", cap)
            ids = torch.empty(2 * Wd * Hd * spp, dtype=torch.int32, device="cuda:0")
            rgb = torch.empty(2 * Wd * Hd * 3, dtype=torch.uint8, device="cuda:0")
            cnt = torch.zeros(2, dtype=torch.int64, device="cuda:0")
            s.frame_stats(0, reset=True)
            s.render_batch_device(0, cams, Wd, Hd, 0, 1, Hd, hit_id=ids.data_ptr(), rgb=rgb.data_ptr(),
                                  hit_count=cnt.data_ptr(), stream=st, spp=spp, count=True)
            torch.cuda.synchronize()
            fs = s.frame_stats(0, reset=True)
            res[cap] = (ids.cpu().numpy().view(np.uint32).reshape(2, -1, spp), rgb.cpu().numpy().reshape(2, -1, 3),
                        cnt.cpu().numpy(), fs["redo_rays"], fs["node_fetches"])
            monkeypatch.delenv("RT_REDO_CAP", raising=False)
        assert res["1"][3] > 1, "the redo list did not overflow"
        # the retry re-traces every pixel without counting: no fetches counted twice
        assert 0 < res["1"][4] <= res[None][4], (res["1"][4], res[None][4])
        for f, (p, d) in enumerate(cams):
            o = ob.render(p, d, Wd, Hd) if spp == 1 else ob.render_spp(p, d, Wd, Hd, spp)
            oid = o["id"].reshape(-1, spp)
            for cap in (None, "1"):
                g = res[cap][0][f]
                assert np.array_equal(np.where(g == rt.RT_MISS, -1, g.astype(np.int64)), oid), (spp, cap, f)
                assert np.array_equal(res[cap][1][f], o["rgb"]), (spp, cap, f)
                assert int(res[cap][2][f]) == o["hits"] > 0, (spp, cap, f)


ARMADILLO = os.environ.get("RT_ARMADILLO_OBJ")


@pytest.mark.skipif(not (ARMADILLO and os.path.exists(ARMADILLO)),
                    reason="armadillo.obj is stripped from the reference; set RT_ARMADILLO_OBJ to run config c3")
def test_armadillo_config_c3(frames_golden, oracle):
    """Config c3's model: the reference's 36 published 500x500 bsah-2 frames
    (testruns_final/testrun_0: PPM sha256, hit counts, camera strings), then
    1920x1080 bsah-8 frames against the oracle."""
    from raytracingdemo_amd.scenes import armadillo_scene
    tris, _ = armadillo_scene()
    g = frames_golden["armadillo.obj"]
    s2 = rt.Scene(tris, "bsah", 2).upload([0])
    path = rt.CameraPath(rt.scene_center(tris), 36)
    for fr in g["frames"]:
        pos, d = path.circular_path(fr["step"])
        assert [f"{v:g}" for v in pos] == fr["cam_pos"]
        out = s2.calculate_screen(pos, d, 500, 500, want=("rgb",))
        assert hashlib.sha256(rt.ppm_bytes(out["rgb"], 500, 500)).hexdigest() == fr["sha256"], fr["step"]
        assert out["hits"] == fr["hits"], fr["step"]
    s8 = rt.Scene(tris, "bsah", 8).upload([0])
    ob = oracle.bvh(tris, "bsah", 8)
    for step in (0, 11, 23):
        pos, d = path.circular_path(step)
        gg = s8.calculate_screen(pos, d, W, H, want=("hit_id", "rgb"))
        o = ob.render(pos, d, W, H, want=("id", "rgb"))
        gid = np.where(gg["hit_id"] == rt.RT_MISS, -1, gg["hit_id"].astype(np.int64))
        assert np.array_equal(gid, o["id"]) and np.array_equal(gg["rgb"], o["rgb"]), step


def test_config_c3_shape_standin_bunny_1080p(oracle):
    """c3-shape stand-in (armadillo stripped): config c3's shape — bsah-8
    k-way, 1920x1080, 1 spp, whole frames — on the largest pinned model
    (stanford-bunny, 69,451 triangles, scale 30), 36-pose orbit in one launch as
    bench.py --scene armadillo would time it; every pixel's id, distance,
    colour and every frame's hit count against the oracle's full frames."""
    tris = golden_scene("stanford-bunny.obj")
    s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    cams = orbit(tris)
    ids, dist, rgb, cnt = render_orbit(s, cams)
    ob = oracle.bvh(tris, "bsah", 8)
    for f in range(0, 36, 5):
        p, d = cams[f]
        o = ob.render(p, d, W, H, want=("id", "dist", "rgb"))
        g_id = ids[f].cpu().numpy().reshape(-1).view(np.uint32)
        gid = np.where(g_id == rt.RT_MISS, -1, g_id.astype(np.int64))
        assert np.array_equal(gid, o["id"]), f
        m = o["id"] >= 0
        assert np.array_equal(dist[f].cpu().numpy().reshape(-1)[m], o["dist"][m]), f
        assert np.array_equal(rgb[f].cpu().numpy().reshape(-1, 3), o["rgb"]), f
        assert int(cnt[f]) == o["hits"] > 0, f


def _paths(s, pos, d, Wp, Hp, frame, spp, bounces, row0, stride, nrows, shadow=False):
    npx = nrows * Wp
    t_id = torch.empty(npx * spp, dtype=torch.int32, device="cuda:0")
    t_dist = torch.empty(npx * spp, dtype=torch.float64, device="cuda:0")
    t_rgb = torch.empty(npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    s.render_paths_device(0, pos, d, Wp, Hp, row0, stride, nrows, frame=frame, spp=spp, bounces=bounces,
                          hit_id=t_id.data_ptr(), dist=t_dist.data_ptr(), rgb=t_rgb.data_ptr(),
                          hit_count=t_cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream,
                          shadow=shadow, count=shadow)
    torch.cuda.synchronize()
    g_id = t_id.cpu().numpy().view(np.uint32).reshape(npx, spp)
    out = {"id": np.where(g_id == rt.RT_MISS, -1, g_id.astype(np.int64)),
           "dist": t_dist.cpu().numpy().reshape(npx, spp), "rgb": t_rgb.cpu().numpy().reshape(npx, 3),
           "hits": int(t_cnt.item())}
    if shadow:
        st = s.frame_stats(0, reset=True)
        out["shadow_cast"], out["shadow_occluded"] = st["shadow_rays"], st["shadow_occluded"]
    return out


def _same_paths(g, o, what):
    assert np.array_equal(g["id"], o["id"]), what
    m = o["id"] >= 0
    assert np.array_equal(g["dist"][m], o["dist"][m]), what
    bad = np.flatnonzero((g["rgb"] != o["rgb"]).any(1))
    assert bad.size == 0, (what, bad[:10])
    assert g["hits"] == o["hits"] > 0, what
    for k in ("shadow_cast", "shadow_occluded"):
        if k in g:
            assert g[k] == o[k], (what, k)


@pytest.mark.parametrize("shadow", [False, True])
def test_config_c5_exact_combination_matches_oracle(oracle, shadow):
    """Config c5 exactly as `bench.py --paths` times it: sponza proxy, walk
    tree built on the device, 3840x2160 camera, 16 spp (the packed path: a
    wave holds every sample of 2x2 pixels), 1 + 4 segments, pose k of the
    orbit with frame = k.  Three bands of 4 full-width rows (top, middle,
    bottom; ~1.1 M segments each) and one strided shard (4 rows 540 apart, the
    row_stride the per-rank call takes) against orc_render_paths: every
    sample's primary id and distance, every pixel's colour and the hit count.
    shadow: with the occlusion rays toward the head-light from every bounce
    vertex (RT_FLAG_SHADOW, as `bench.py --paths` times it), also the numbers
    of occlusion rays cast and occluded.
    Reference: StackBVH::traverse per segment (src/stack_bvh.hpp:611-644),
    the vertex colour of shadeScreen (src/main.cpp:356-377)."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    ob = oracle.bvh(tris, "bsah", 8)
    Wp, Hp, S, B = 3840, 2160, 16, 4
    path = rt.CameraPath(rt.scene_center(tris), 36)
    for frame in (0, 1):
        pos, d = path.circular_path(frame)
        for row0 in (0, Hp // 2 - 2, Hp - 4):
            g = _paths(s, pos, d, Wp, Hp, frame, S, B, row0, 1, 4, shadow)
            o = ob.render_paths(pos, d, Wp, Hp, frame, S, B, row0=row0, nrows=4, shadow=shadow)
            _same_paths(g, o, (frame, row0))
    # a strided shard (rows 3, 543, 1083, 1623: row0 = rank, stride = world)
    pos, d = path.circular_path(2)
    g = _paths(s, pos, d, Wp, Hp, 2, S, B, 3, 540, 4, shadow)
    parts = [ob.render_paths(pos, d, Wp, Hp, 2, S, B, row0=r, nrows=1, shadow=shadow) for r in (3, 543, 1083, 1623)]
    o = {k: np.concatenate([p[k] for p in parts]) for k in ("id", "dist", "rgb")}
    for k in ("hits", "shadow_cast", "shadow_occluded"):
        o[k] = sum(p[k] for p in parts)
    _same_paths(g, o, "strided shard")


def test_config_c5_full_pose_one_call_matches_oracle(oracle):
    """Config c5 at its timed shape: ONE rt_render_paths_device call over the
    whole 3840x2160 pose at 16 spp x (1 + 4) segments with the head-light
    occlusion rays, exactly as `bench.py --paths` times it (132.7 M paths,
    ~410 M sorted occlusion records, the 8-way partitioned queues, the 3-pass
    key sort across RT_SH_BLOCKS) — against orc_render_paths over every row of
    the pose: every sample's primary hit id and distance, every pixel's colour,
    the pose's hit count, and (from a counting render of the same call, whose
    colours must equal the timed one's) the occlusion rays cast and occluded.
    The oracle runs in bands of rows on the host's cores (~35 s at 16).
    Reference: StackBVH::traverse per segment (src/stack_bvh.hpp:611-644),
    the vertex colour of shadeScreen (src/main.cpp:356-377)."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    Wp, Hp, S, B, frame = 3840, 2160, 16, 4, 5
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(frame)
    npx = Wp * Hp
    t_id = torch.empty(npx * S, dtype=torch.int32, device="cuda:0")
    t_dist = torch.empty(npx * S, dtype=torch.float64, device="cuda:0")
    t_rgb = torch.empty(npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.full((1,), 12345, dtype=torch.int64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream

    def call(rgb, count, store):
        s.render_paths_device(0, pos, d, Wp, Hp, 0, 1, Hp, frame=frame, spp=S, bounces=B, hit_id=t_id.data_ptr(),
                              dist=t_dist.data_ptr(), rgb=rgb.data_ptr(), hit_count=t_cnt.data_ptr(), stream=st,
                              shadow=True, count=count, counts_store=store)

    call(t_rgb, False, True)  # the timed call (RT_FLAG_COUNTS_STORE: the stale 12345 is replaced)
    torch.cuda.synchronize()
    hits = int(t_cnt.item())
    rgb2 = torch.empty_like(t_rgb)
    s.frame_stats(0, reset=True)
    call(rgb2, True, True)
    torch.cuda.synchronize()
    fs = s.frame_stats(0, reset=True)
    assert torch.equal(rgb2, t_rgb) and int(t_cnt.item()) == hits
    g_id = t_id.cpu().numpy().view(np.uint32).reshape(Hp, Wp * S)
    g_dist = t_dist.cpu().numpy().reshape(Hp, Wp * S)
    g_rgb = t_rgb.cpu().numpy().reshape(Hp, Wp * 3)
    ob = oracle.bvh(tris, "bsah", 8)
    o_hits = o_cast = o_occ = 0
    band = 120
    for r0 in range(0, Hp, band):
        o = ob.render_paths(pos, d, Wp, Hp, frame, S, B, row0=r0, nrows=band, shadow=True)
        gid = g_id[r0:r0 + band].reshape(-1, S)
        gid = np.where(gid == rt.RT_MISS, -1, gid.astype(np.int64))
        assert np.array_equal(gid, o["id"]), (r0, np.flatnonzero((gid != o["id"]).any(1))[:8])
        m = o["id"] >= 0
        assert np.array_equal(g_dist[r0:r0 + band].reshape(-1, S)[m], o["dist"][m]), r0
        bad = np.flatnonzero((g_rgb[r0:r0 + band].reshape(-1, 3) != o["rgb"]).any(1))
        assert bad.size == 0, (r0, bad[:10])
        o_hits += o["hits"]
        o_cast += o["shadow_cast"]
        o_occ += o["shadow_occluded"]
    assert hits == o_hits > 0
    assert fs["shadow_rays"] == o_cast > 0 and fs["shadow_occluded"] == o_occ
    print(f"\nc5 full pose: {hits} primary hits, {o_cast} occlusion rays ({o_occ} occluded)")


@pytest.mark.parametrize("model", ["sponza-proxy", "stanford-bunny.obj", "teapot.obj", "suzanne.obj", "dup-stack"])
def test_device_walk_tree_build(oracle, model):
    """The walk tree built on the device (rt_scene_create_on_device) makes the
    host builder's splits: the same wide-node count and stack bound on scenes
    without positional splits, and frames identical to the oracle's."""
    if model == "sponza-proxy":
        from raytracingdemo_amd.scenes import sponza_proxy_triangles
        tris, algo = sponza_proxy_triangles(), "bsah"
    elif model == "dup-stack":
        tris, algo = _dup_stack(40), "sah"  # coincident centroids: positional splits
    else:
        tris, algo = golden_scene(model), "bsah"
    host = rt.Scene(tris, algo, 8)
    dev = rt.Scene(tris, algo, 8, walk_device=0)
    bt = dev.build_times()
    assert bt["walk_device"] == 0 and host.build_times()["walk_device"] == -1
    hs, ds = host.stats(), dev.stats()
    assert ds["walk_tree"] == 1 and ds["triangles"] == hs["triangles"]
    if model != "dup-stack":
        assert ds["wide_nodes"] == hs["wide_nodes"] and ds["stack_bound"] == hs["stack_bound"], (hs, ds)
    dev.upload([0])
    path = rt.CameraPath(rt.scene_center(tris), 36)
    W, H = (1920, 1080) if model == "sponza-proxy" else (320, 240)
    ob = oracle.bvh(tris, algo, 8)
    for step in (0, 17) if model != "dup-stack" else (0,):
        pos, d = path.circular_path(step) if model != "dup-stack" else ([0.0, 0.0, 3.0], [0.0, 0.0, -1.0])
        g = dev.calculate_screen(pos, d, W, H, want=("hit_id", "dist", "rgb"))
        o = ob.render(pos, d, W, H, want=("id", "dist", "rgb"))
        gid = np.where(g["hit_id"] == rt.RT_MISS, -1, g["hit_id"].astype(np.int64))
        assert np.array_equal(gid, o["id"]), (model, step)
        m = o["id"] >= 0
        assert np.array_equal(g["dist"][m], o["dist"][m]) and np.array_equal(g["rgb"], o["rgb"]), (model, step)
    print(f"\n{model}: walk tree host {host.build_times()['walk_tree_ms']:.1f} ms, device {bt['walk_tree_ms']:.1f} ms")
