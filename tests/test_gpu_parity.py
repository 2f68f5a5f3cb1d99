"""GPU parity: the gfx950 kernels through the C ABI vs the reference's goldens
and the oracle.  Bit-exact hit-IDs, hit positions (fp64), distances and PPM
bytes; both traversal modes (exact-fast and literal fp64)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import golden_scene, normals_of, pixel_fixture, pixel_fixture_names

pytestmark = pytest.mark.gpu

rt = pytest.importorskip("raytracingdemo_amd")
MODELS = ["teapot.obj", "suzanne.obj", "stanford-bunny.obj"]
_SCENES: dict = {}


def scene(model, algo="bsah", k=2, scale=None, tris=None):
    key = (model, algo, k, scale)
    if key not in _SCENES:
        t = golden_scene(model, scale) if tris is None else tris
        _SCENES[key] = rt.Scene(t, algo, k).upload([0])
    return _SCENES[key]


def compare_with_oracle(oracle, s, tris, pos, d, W, H, algo, k, mode="exact"):
    g = s.calculate_screen(pos, d, W, H, mode=mode)
    o = oracle.bvh(tris, algo, k).render(pos, d, W, H)
    oid = o["id"].astype(np.int64)
    gid = np.where(g["hit_id"] == rt.RT_MISS, -1, g["hit_id"].astype(np.int64))
    assert np.array_equal(gid, oid), f"hit-id mismatch at {np.flatnonzero(gid != oid)[:10]}"
    m = oid >= 0
    assert np.array_equal(g["pos"][m], o["pos"][m])
    assert np.array_equal(g["dist"][m], o["dist"][m])
    assert np.all(g["dist"][~m] == -1.0)
    assert np.array_equal(g["rgb"], o["rgb"])
    assert g["hits"] == o["hits"]
    return g


@pytest.mark.parametrize("mode", ["exact", "fp64"])
@pytest.mark.parametrize("model", MODELS)
def test_reference_frames_bit_exact(frames_golden, model, mode):
    """500x500 frames 0,9,17,27 == testruns_final PPM bytes and hit counts
    (one set of host arrays reused across the frames, as runTest does)."""
    g = frames_golden[model]
    tris = golden_scene(model)
    s = scene(model, "bsah", 2)
    c = rt.scene_center(tris)
    out = None
    for step in (0, 9, 17, 27):
        pos, d = rt.CameraPath(c, 36).circular_path(step)
        out = s.calculate_screen(pos, d, 500, 500, mode=mode, want=("rgb",), out=out)
        assert hashlib.sha256(rt.ppm_bytes(out["rgb"], 500, 500)).hexdigest() == g["frames"][step]["sha256"], step
        assert out["hits"] == g["frames"][step]["hits"]


@pytest.mark.parametrize("algo,k", [("bsah", 4), ("bsah", 8), ("bsah", 16), ("sah", 4), ("median", 16),
                                    ("bsah-c", 8), ("sah-c", 16), ("median-c", 4)])
def test_every_tree_variant_gives_reference_frame(frames_golden, algo, k):
    """The reference's validate_data invariant: identical bytes for every BVH."""
    for model in MODELS:
        tris = golden_scene(model)
        s = scene(model, algo, k)
        c = rt.scene_center(tris)
        step = 17
        pos, d = rt.CameraPath(c, 36).circular_path(step)
        out = s.calculate_screen(pos, d, 500, 500, want=("rgb",))
        assert hashlib.sha256(rt.ppm_bytes(out["rgb"], 500, 500)).hexdigest() == \
            frames_golden[model]["frames"][step]["sha256"], (model, algo, k)


@pytest.mark.parametrize("name", pixel_fixture_names())
def test_pixels_vs_reference_fixture(name):
    """Per-pixel fixtures produced by the compiled reference (oracle/_ref)."""
    z = pixel_fixture(name)
    model = str(z["model"])
    tris = golden_scene(model, float(z["scale"]))
    s = scene(model, str(z["algo"]), int(z["k"]), float(z["scale"]), tris)
    W, H = int(z["W"]), int(z["H"])
    g = s.calculate_screen(z["cam_pos"], z["cam_dir"], W, H)
    hit = np.unpackbits(z["hit"])[: W * H].astype(bool)
    assert np.array_equal(g["hit_id"] != rt.RT_MISS, hit)
    assert np.array_equal(g["rgb"], z["rgb"])
    assert g["hits"] == int(z["hits"])
    sel = z["sel"]
    hs = hit[sel]
    assert np.array_equal(g["pos"][sel][hs], z["pos"][hs])
    nrm = normals_of(tris)[g["hit_id"][sel][hs].astype(np.int64)]
    assert np.array_equal(nrm, z["nrm"][hs])


@pytest.mark.parametrize("mode", ["exact", "fp64"])
def test_vs_oracle_random_cameras(oracle, mode):
    rng = np.random.default_rng(1234)
    for model, algo, k in [("teapot.obj", "bsah", 8), ("suzanne.obj", "sah-c", 8), ("stanford-bunny.obj", "median", 2)]:
        tris = golden_scene(model)
        s = scene(model, algo, k)
        c = rt.scene_center(tris)
        lo, hi = tris.reshape(-1, 3).min(0), tris.reshape(-1, 3).max(0)
        for _ in range(3):
            pos = c + rng.uniform(-1.0, 1.0, 3) * (hi - lo) * 1.2
            d = c + rng.uniform(-0.3, 0.3, 3) * (hi - lo) - pos
            d = d / np.sqrt((d * d).sum())
            W, H = int(rng.integers(16, 160)), int(rng.integers(16, 120))
            compare_with_oracle(oracle, s, tris, pos, d, W, H, algo, k, mode)


def test_non_square_and_odd_sizes(oracle):
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 4)
    c = rt.scene_center(tris)
    pos, d = rt.CameraPath(c, 36).circular_path(4)
    for W, H in [(1, 1), (7, 3), (640, 360), (123, 457), (1920, 1080)]:
        compare_with_oracle(oracle, s, tris, pos, d, W, H, "bsah", 4)


def test_sponza_proxy_bands_vs_oracle(oracle):
    """Headline scene (262,267-triangle proxy), 1920x1080 BVH8: row bands vs oracle."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    c = rt.scene_center(tris)
    b = oracle.bvh(tris, "bsah", 8)
    for step in (0, 13, 29):
        pos, d = rt.CameraPath(c, 36).circular_path(step)
        g = s.calculate_screen(pos, d, 1920, 1080)
        for row0 in (0, 389, 777, 1064):
            o = b.render(pos, d, 1920, 1080, row0=row0, nrows=16)
            sl = slice(row0 * 1920, (row0 + 16) * 1920)
            gid = np.where(g["hit_id"][sl] == rt.RT_MISS, -1, g["hit_id"][sl].astype(np.int64))
            assert np.array_equal(gid, o["id"]), (step, row0)
            m = o["id"] >= 0
            assert np.array_equal(g["pos"][sl][m], o["pos"][m])
            assert np.array_equal(g["rgb"][sl], o["rgb"])


@pytest.mark.parametrize("env", [{"RT_WALK_COLLAPSE": "greedy"}, {"RT_WALK_CN": "2"}, {"RT_WALK_LEAF": "1"}])
def test_walk_tree_collapse_variants_give_identical_frames(env, monkeypatch):
    """Results never depend on the walk tree (walk_tree.cpp): the greedy
    collapse, a costlier node visit in the collapse and one-triangle binary leaves render
    the headline scene's frames bit for bit like the default planned collapse
    (the full-size test in test_gpu_headline.py pins the default to the oracle)."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    c = rt.scene_center(tris)
    base = rt.Scene(tris, "bsah", 8).upload([0])
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alt = rt.Scene(tris, "bsah", 8).upload([0])
    assert alt.stats()["layout_digest"] != base.stats()["layout_digest"]
    for step in (3, 21):
        pos, d = rt.CameraPath(c, 36).circular_path(step)
        x = base.calculate_screen(pos, d, 960, 540)
        y = alt.calculate_screen(pos, d, 960, 540)
        for f in ("hit_id", "pos", "dist", "rgb"):
            assert np.array_equal(x[f], y[f]), (env, step, f)
        assert x["hits"] == y["hits"]


def test_exact_and_literal_modes_agree_on_sponza_proxy():
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles(60000)
    s = rt.Scene(tris, "bsah", 8).upload([0])
    c = rt.scene_center(tris)
    pos, d = rt.CameraPath(c, 36).circular_path(7)
    a = s.calculate_screen(pos, d, 320, 180, mode="exact")
    b = s.calculate_screen(pos, d, 320, 180, mode="fp64")
    for key in ("hit_id", "dist", "pos", "rgb"):
        assert np.array_equal(a[key], b[key]), key


def test_distance_ties_resolve_in_reference_visit_order(oracle):
    """Coincident duplicate triangles tie exactly; the reference keeps the first
    one it visits (strict '<', stack_bvh.hpp:631)."""
    base = golden_scene("suzanne.obj")
    tris = np.concatenate([base, base[::7]])  # duplicates of every 7th triangle
    for algo, k in [("sah", 2), ("median", 8), ("sah-c", 16)]:
        s = rt.Scene(tris, algo, k).upload([0])
        c = rt.scene_center(tris)
        pos, d = rt.CameraPath(c, 36).circular_path(3)
        compare_with_oracle(oracle, s, tris, pos, d, 160, 120, algo, k)
        compare_with_oracle(oracle, s, tris, pos, d, 160, 120, algo, k, mode="fp64")


def test_edge_scenes(oracle):
    # empty scene: every ray misses
    s = rt.Scene(np.zeros((0, 9)), "bsah", 8).upload([0])
    out = s.calculate_screen([0, 0, 5], [0, 0, -1], 32, 16)
    assert out["hits"] == 0 and np.all(out["hit_id"] == rt.RT_MISS) and not out["rgb"].any()
    # one triangle, leaf root
    tri = np.array([[-1.0, -1.0, 0.0, 1.0, -1.0, 0.0, 0.0, 1.0, 0.0]])
    s = rt.Scene(tri, "bsah", 2).upload([0])
    compare_with_oracle(oracle, s, tri, [0.0, 0.0, 3.0], [0.0, 0.0, -1.0], 64, 48, "bsah", 2)
    # camera looking away from the scene: all miss (boxes behind the camera are
    # still "hit" by the reference's unclipped slab test, but no triangle is)
    tris = golden_scene("teapot.obj")
    s = scene("teapot.obj", "bsah", 8)
    c = rt.scene_center(tris)
    out = s.calculate_screen(c + np.array([0.0, 0.0, 8.0]), [0.0, 0.0, 1.0], 64, 64)
    assert out["hits"] == 0
    # degenerate (zero-area) triangles never hit (|a| < EPS, triangle.hpp:46)
    deg = np.concatenate([tris[:100], np.tile(tris[:1, 0:3], (1, 3))])
    s = rt.Scene(deg, "sah", 4).upload([0])
    compare_with_oracle(oracle, s, deg, c + np.array([0.0, 0.0, 5.0]), [0.0, 0.0, -1.0], 80, 60, "sah", 4)


def _stack_scene(eps: float, n: int, far_hit: bool) -> np.ndarray:
    """n triangles stacked along -z with a corner at (eps, eps): the centre ray
    of an odd-sized frame (direction exactly (0, 0, -1)) grazes every corner,
    so the fp32 filter can only call them borderline."""
    tris = [[eps, eps, -k, 1.0, eps, -k, eps, 1.0, -k] for k in range(1, n + 1)]
    if far_hit:  # one robust hit far behind the stack
        z = -float(n + 16)
        tris.append([-3.0, -3.0, z, 3.0, -3.0, z, 0.0, 3.0, z])
    return np.array(tris, dtype=np.float64)


def test_candidate_overflow_paths(oracle):
    """More borderline candidates than the per-lane LDS list holds (8): the
    next 24 go to the lane's overflow pool chunk, past those they are dropped.

    (a) corners exactly on the ray: the nearest is a real hit (certified
        against the smallest dropped bound when there are > 32);
    (b) corners 1e-7 off the ray: every listed candidate fails the exact test;
        with 14 the real hit is still in the pool chunk (no redo), with 40
        it was dropped, so the pixel must be redone by the fix-up kernel.
    All must equal the reference traversal."""
    torch = pytest.importorskip("torch")
    for eps, n, far, need_redo in ((0.0, 14, False, False), (1e-7, 14, True, False),
                                   (0.0, 40, False, False), (1e-7, 40, True, True)):
        tris = _stack_scene(eps, n, far)
        s = rt.Scene(tris, "bsah", 8).upload([0])
        for W in (33, 65):
            compare_with_oracle(oracle, s, tris, [0.0, 0.0, 10.0], [0.0, 0.0, -1.0], W, W, "bsah", 8)
        W = 33
        ids = torch.empty(W * W, dtype=torch.int32, device="cuda:0")
        st = torch.cuda.current_stream()
        s.frame_stats(0, reset=True)
        s.render_rows_device(0, [0.0, 0.0, 10.0], [0.0, 0.0, -1.0], W, W, 0, 1, W, hit_id=ids.data_ptr(),
                             stream=st.cuda_stream, count=True)
        torch.cuda.synchronize()
        fs = s.frame_stats(0, reset=True)
        # redo because of the bounded list (not because the reference cannot
        # see the winner: with d = (0, 0, -1) the reference's (0 - 0) * inf slab
        # terms are NaN, and chain failures are expected on the corner pixel)
        over = fs["redo_rays"] - fs["redo_chain"]
        assert (over > 0) == need_redo, (fs["redo_rays"], fs["redo_chain"])


def test_row_shards_reassemble_to_full_frame():
    """Row-interleaved shards (multi-GPU partition) rebuild the full frame bit for bit."""
    torch = pytest.importorskip("torch")
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 4)
    c = rt.scene_center(tris)
    pos, d = rt.CameraPath(c, 36).circular_path(11)
    W, H = 320, 240
    full = s.calculate_screen(pos, d, W, H)
    for G in (2, 3, 8):
        rgb = np.zeros((H, W, 3), np.uint8)
        ids = np.zeros((H, W), np.uint32)
        hits = 0
        for r in range(G):
            nrows = len(range(r, H, G))
            t_id = torch.empty(nrows * W, dtype=torch.int32, device="cuda:0")
            t_rgb = torch.empty(nrows * W * 3, dtype=torch.uint8, device="cuda:0")
            t_cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
            st = torch.cuda.current_stream()
            s.render_rows_device(0, pos, d, W, H, r, G, nrows, hit_id=t_id.data_ptr(), rgb=t_rgb.data_ptr(),
                                 hit_count=t_cnt.data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize()
            ids[r::G] = t_id.cpu().numpy().view(np.uint32).reshape(nrows, W)
            rgb[r::G] = t_rgb.cpu().numpy().reshape(nrows, W, 3)
            hits += int(t_cnt.item())
        assert np.array_equal(ids.reshape(-1), full["hit_id"])
        assert np.array_equal(rgb.reshape(-1, 3), full["rgb"])
        assert hits == full["hits"]


@pytest.mark.parametrize("mode", ["exact", "fp64"])
def test_batched_frames_equal_single_frames(mode):
    """rt_render_batch_device over 27 poses (one launch; up to 36 poses fit
    one) of a row shard equals 27 single-frame renders: ids, distances,
    positions, colours and per-frame hit counts, bit for bit."""
    torch = pytest.importorskip("torch")
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(0, 36, 1)][:27]
    W, H, row0, stride = 150, 101, 1, 2
    nrows = len(range(row0, H, stride))
    F, npx = len(cams), nrows * W
    t_id = torch.empty(F * npx, dtype=torch.int32, device="cuda:0")
    t_dist = torch.empty(F * npx, dtype=torch.float64, device="cuda:0")
    t_pos = torch.empty(F * npx * 3, dtype=torch.float64, device="cuda:0")
    t_rgb = torch.empty(F * npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    st = torch.cuda.current_stream()
    s.render_batch_device(0, cams, W, H, row0, stride, nrows, hit_id=t_id.data_ptr(), dist=t_dist.data_ptr(),
                          hit_pos=t_pos.data_ptr(), rgb=t_rgb.data_ptr(), hit_count=t_cnt.data_ptr(),
                          stream=st.cuda_stream, mode=mode)
    torch.cuda.synchronize()
    ids = t_id.cpu().numpy().view(np.uint32).reshape(F, nrows, W)
    dist = t_dist.cpu().numpy().reshape(F, nrows, W)
    pos = t_pos.cpu().numpy().reshape(F, nrows, W, 3)
    rgb = t_rgb.cpu().numpy().reshape(F, nrows, W, 3)
    cnt = t_cnt.cpu().numpy()
    for f, (p, d) in enumerate(cams):
        g = s.calculate_screen(p, d, W, H, mode=mode)
        sl = slice(row0, H, stride)
        assert np.array_equal(ids[f], g["hit_id"].reshape(H, W)[sl]), f
        assert np.array_equal(dist[f], g["dist"].reshape(H, W)[sl]), f
        hit = ids[f] != rt.RT_MISS
        assert np.array_equal(pos[f][hit], g["pos"].reshape(H, W, 3)[sl][hit]), f
        assert np.array_equal(rgb[f], g["rgb"].reshape(H, W, 3)[sl]), f
        assert cnt[f] == int(hit.sum()), f
    assert cnt.sum() > 0


def test_batched_frames_on_sponza_proxy_match_the_oracle(oracle):
    """A 12-pose batch (one launch) of sponza-proxy bands against the oracle."""
    torch = pytest.importorskip("torch")
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    ob = oracle.bvh(tris, "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(0, 36, 3)]
    W, H, row0, stride = 192, 108, 0, 9  # every 9th row of a 192x108 image
    nrows = len(range(row0, H, stride))
    F, npx = len(cams), nrows * W
    t_id = torch.empty(F * npx, dtype=torch.int32, device="cuda:0")
    t_rgb = torch.empty(F * npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, row0, stride, nrows, hit_id=t_id.data_ptr(), rgb=t_rgb.data_ptr(),
                          hit_count=t_cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ids = t_id.cpu().numpy().view(np.uint32).reshape(F, nrows, W)
    rgb = t_rgb.cpu().numpy().reshape(F, nrows, W, 3)
    for f, (p, d) in enumerate(cams):
        o = ob.render(p, d, W, H)
        oid = o["id"].reshape(H, W)[row0::stride]
        gid = np.where(ids[f] == rt.RT_MISS, -1, ids[f].astype(np.int64))
        assert np.array_equal(gid, oid), f
        assert np.array_equal(rgb[f], o["rgb"].reshape(H, W, 3)[row0::stride]), f


def _spp_render(s, cams, W, H, spp, row0=0, stride=1, nrows=None, mode="exact"):
    torch = pytest.importorskip("torch")
    nrows = len(range(row0, H, stride)) if nrows is None else nrows
    F, npx = len(cams), nrows * W
    t_id = torch.empty(F * npx * spp, dtype=torch.int32, device="cuda:0")
    t_dist = torch.empty(F * npx * spp, dtype=torch.float64, device="cuda:0")
    t_pos = torch.empty(F * npx * spp * 3, dtype=torch.float64, device="cuda:0")
    t_rgb = torch.empty(F * npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, row0, stride, nrows, hit_id=t_id.data_ptr(), dist=t_dist.data_ptr(),
                          hit_pos=t_pos.data_ptr(), rgb=t_rgb.data_ptr(), hit_count=t_cnt.data_ptr(),
                          stream=torch.cuda.current_stream().cuda_stream, mode=mode, spp=spp)
    torch.cuda.synchronize()
    return {"id": t_id.cpu().numpy().view(np.uint32).reshape(F, npx, spp),
            "dist": t_dist.cpu().numpy().reshape(F, npx, spp), "pos": t_pos.cpu().numpy().reshape(F, npx, spp, 3),
            "rgb": t_rgb.cpu().numpy().reshape(F, npx, 3), "hits": t_cnt.cpu().numpy()}


@pytest.mark.parametrize("mode", ["exact", "fp64", "split"])
@pytest.mark.parametrize("spp", [4, 9, 16])
def test_stratified_spp_matches_oracle(oracle, spp, mode, monkeypatch):
    """spp = n*n stratified samples per pixel (config c4's 2x2, a 3x3 and a
    4x4): every sample's hit id, distance and position, the averaged colour and
    the per-pose hit count against the oracle; 5 poses span launch boundaries.
    "exact" is the fused resolve (spp 4 and 16: a wave takes all samples of
    4x4 / 2x2 pixels and sums them across its lanes; spp 9: one sample frame
    per tile, k_average forming the pixels), "split" the candidate lists
    handed to k_resolve."""
    if spp == 16 and mode != "exact":
        pytest.skip("16 spp: the fused, packed path only")
    if mode == "split":
        monkeypatch.setenv("RT_RESOLVE", "split")
        mode = "exact"
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    b = oracle.bvh(tris, "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (0, 7, 14, 21, 29)]
    W, H = 96, 64
    g = _spp_render(s, cams, W, H, spp, mode=mode)
    for f, (p, d) in enumerate(cams):
        o = b.render_spp(p, d, W, H, spp)
        gid = np.where(g["id"][f] == rt.RT_MISS, -1, g["id"][f].astype(np.int64))
        assert np.array_equal(gid, o["id"]), f
        m = o["id"] >= 0
        assert np.array_equal(g["dist"][f][m], o["dist"][m]), f
        assert np.all(g["dist"][f][~m] == -1.0)
        assert np.array_equal(g["pos"][f][m], o["pos"][m]), f
        assert np.array_equal(g["rgb"][f], o["rgb"]), f
        assert g["hits"][f] == o["hits"], f


@pytest.mark.parametrize("spp", [4, 16])
def test_packed_samples_equal_sample_frames(spp, monkeypatch):
    """A wave holding every sample of (8/n)^2 pixels (fp.pack, packet_kernel.h)
    renders what one-sample-frame-per-tile tiles and k_average render, bit for
    bit, on odd frame sizes (partial tiles) and a strided row shard."""
    tris = golden_scene("suzanne.obj")
    s = scene("suzanne.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (3, 17, 30)]
    for W, H, row0, stride in [(37, 23, 0, 1), (64, 48, 1, 3)]:
        monkeypatch.setenv("RT_SPP_PACK", "0")
        a = _spp_render(s, cams, W, H, spp, row0=row0, stride=stride)
        monkeypatch.delenv("RT_SPP_PACK")
        b = _spp_render(s, cams, W, H, spp, row0=row0, stride=stride)
        for k in ("id", "dist", "pos", "rgb", "hits"):
            assert np.array_equal(a[k], b[k]), (spp, W, H, k)


def test_spp_row_shards_and_sponza_band(oracle):
    """4 spp on the sponza proxy: a strided row shard equals the same rows of
    the full render, and a row band equals the oracle."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (4, 22)]
    W, H = 160, 90
    full = _spp_render(s, cams, W, H, 4)
    sh = _spp_render(s, cams, W, H, 4, row0=2, stride=3)
    rows = list(range(2, H, 3))
    for f in range(len(cams)):
        fi = full["id"][f].reshape(H, W, 4)[rows].reshape(-1, 4)
        assert np.array_equal(sh["id"][f], fi), f
        assert np.array_equal(sh["rgb"][f], full["rgb"][f].reshape(H, W, 3)[rows].reshape(-1, 3)), f
    b = oracle.bvh(tris, "bsah", 8)
    for f, (p, d) in enumerate(cams):
        o = b.render_spp(p, d, W, H, 4, row0=30, nrows=20)
        gid = full["id"][f].reshape(H, W, 4)[30:50].reshape(-1, 4)
        assert np.array_equal(np.where(gid == rt.RT_MISS, -1, gid.astype(np.int64)), o["id"]), f
        assert np.array_equal(full["rgb"][f].reshape(H, W, 3)[30:50].reshape(-1, 3), o["rgb"]), f


def test_spp_one_equals_the_reference_path():
    """spp = 1 through the multi-sample entry point is the reference path."""
    tris = golden_scene("teapot.obj")
    s = scene("teapot.obj", "bsah", 4)
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(5)
    g = _spp_render(s, [(pos, d)], 80, 60, 1)
    ref = s.calculate_screen(pos, d, 80, 60)
    assert np.array_equal(g["id"][0][:, 0], ref["hit_id"])
    assert np.array_equal(g["rgb"][0], ref["rgb"])
    assert g["hits"][0] == ref["hits"]


def _paths_render(s, pos, d, W, H, frame, spp, bounces, row0=0, stride=1, shadow=False, stats=False):
    torch = pytest.importorskip("torch")
    nrows = len(range(row0, H, stride))
    npx = nrows * W
    t_id = torch.empty(npx * spp, dtype=torch.int32, device="cuda:0")
    t_dist = torch.empty(npx * spp, dtype=torch.float64, device="cuda:0")
    t_rgb = torch.empty(npx * 3, dtype=torch.uint8, device="cuda:0")
    t_cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    s.render_paths_device(0, pos, d, W, H, row0, stride, nrows, frame=frame, spp=spp, bounces=bounces,
                          hit_id=t_id.data_ptr(), dist=t_dist.data_ptr(), rgb=t_rgb.data_ptr(),
                          hit_count=t_cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream,
                          shadow=shadow, count=stats)
    torch.cuda.synchronize()
    out = {"id": t_id.cpu().numpy().view(np.uint32).reshape(npx, spp), "dist": t_dist.cpu().numpy().reshape(npx, spp),
           "rgb": t_rgb.cpu().numpy().reshape(npx, 3), "hits": int(t_cnt.item())}
    if stats:
        out["stats"] = s.frame_stats(0, reset=True)
    return out


@pytest.mark.parametrize("model,spp,bounces,shadow", [("stanford-bunny.obj", 4, 4, False), ("suzanne.obj", 3, 2, False),
                                                      ("teapot.obj", 1, 0, False), ("stanford-bunny.obj", 16, 2, False),
                                                      ("stanford-bunny.obj", 4, 4, True), ("suzanne.obj", 3, 2, True),
                                                      ("teapot.obj", 16, 3, True)])
def test_paths_match_oracle(oracle, model, spp, bounces, shadow):
    """Diffuse paths (secondary rays, config c5's model at small size): every
    pixel colour, every sample's primary hit and the hit count equal the oracle;
    bounces = 0 with one sample is a jittered primary render.  spp 4 and 16
    run packed (a wave holds every sample of 16 / 4 pixels, path_kernel.h).
    shadow: occlusion rays toward the head-light at every bounce vertex
    (RT_FLAG_SHADOW; the oracle's occluded()), cast and occluded counts too."""
    tris = golden_scene(model)
    s = scene(model, "bsah", 8)
    b = oracle.bvh(tris, "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    W, H = 72, 40
    for frame in (2, 19):
        pos, d = path.circular_path(frame)
        g = _paths_render(s, pos, d, W, H, frame, spp, bounces, shadow=shadow, stats=shadow)
        o = b.render_paths(pos, d, W, H, frame, spp, bounces, shadow=shadow)
        if shadow:
            assert g["stats"]["shadow_rays"] == o["shadow_cast"], frame
            assert g["stats"]["shadow_occluded"] == o["shadow_occluded"], frame
        gid = np.where(g["id"] == rt.RT_MISS, -1, g["id"].astype(np.int64))
        assert np.array_equal(gid, o["id"]), frame
        m = o["id"] >= 0
        assert np.array_equal(g["dist"][m], o["dist"][m]), frame
        assert np.array_equal(g["rgb"], o["rgb"]), (frame, np.flatnonzero((g["rgb"] != o["rgb"]).any(1))[:10])
        assert g["hits"] == o["hits"], frame
        assert g["rgb"].max() > 0


@pytest.mark.parametrize("spp", [2, 8, 16, 32])
def test_paths_packed_equal_per_lane_samples(spp, monkeypatch):
    """k_paths with every sample of 64 / spp pixels in one wave (one path per
    lane, the radiance summed across lanes) equals one pixel per lane with
    its samples in a loop, bit for bit: odd sizes, a strided shard."""
    tris = golden_scene("suzanne.obj")
    s = scene("suzanne.obj", "bsah", 8)
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(11)
    for W, H, row0, stride in [(37, 23, 0, 1), (50, 31, 2, 3)]:
        monkeypatch.setenv("RT_PATHS_PACK", "0")
        a = _paths_render(s, pos, d, W, H, 11, spp, 3, row0, stride)
        monkeypatch.delenv("RT_PATHS_PACK")
        b = _paths_render(s, pos, d, W, H, 11, spp, 3, row0, stride)
        for k in ("id", "dist", "rgb", "hits"):
            assert np.array_equal(a[k], b[k]), (spp, W, H, k)
        assert b["rgb"].max() > 0


def test_paths_sponza_proxy_shard(oracle):
    """Paths on the sponza proxy: a strided row shard equals those rows of the
    full render, and a row band equals the oracle (4 samples, 4 bounces)."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8).upload([0])
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(11)
    W, H = 96, 54
    full = _paths_render(s, pos, d, W, H, 11, 4, 4)
    sh = _paths_render(s, pos, d, W, H, 11, 4, 4, row0=1, stride=4)
    rows = list(range(1, H, 4))
    assert np.array_equal(sh["rgb"], full["rgb"].reshape(H, W, 3)[rows].reshape(-1, 3))
    o = oracle.bvh(tris, "bsah", 8).render_paths(pos, d, W, H, 11, 4, 4, row0=20, nrows=12)
    assert np.array_equal(full["rgb"].reshape(H, W, 3)[20:32].reshape(-1, 3), o["rgb"])
    gid = full["id"].reshape(H, W, 4)[20:32].reshape(-1, 4)
    assert np.array_equal(np.where(gid == rt.RT_MISS, -1, gid.astype(np.int64)), o["id"])


def test_paths_shadow_sponza_proxy_band(oracle):
    """Occlusion rays on the sponza proxy (the scene where they matter: most
    bounce vertices are hidden from the camera): a 16-spp 4-bounce row band
    and a strided shard equal the oracle — colours, primary ids, hit count, and
    the numbers of occlusion rays cast and occluded."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    s = rt.Scene(tris, "bsah", 8, walk_device=0).upload([0])
    ob = oracle.bvh(tris, "bsah", 8)
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(5)
    W, H = 320, 180
    g = _paths_render(s, pos, d, W, H, 5, 16, 4, row0=60, stride=1, shadow=True, stats=True)
    g_id = np.where(g["id"] == rt.RT_MISS, -1, g["id"].astype(np.int64))
    full = ob.render_paths(pos, d, W, H, 5, 16, 4, shadow=True)
    assert np.array_equal(g["rgb"], full["rgb"][60 * W:]), np.flatnonzero((g["rgb"] != full["rgb"][60 * W:]).any(1))[:10]
    assert np.array_equal(g_id, full["id"][60 * W:])
    o = ob.render_paths(pos, d, W, H, 5, 16, 4, row0=60, shadow=True)
    assert g["hits"] == o["hits"] > 0
    assert g["stats"]["shadow_rays"] == o["shadow_cast"] > 0
    assert g["stats"]["shadow_occluded"] == o["shadow_occluded"] > 0
    sh = _paths_render(s, pos, d, W, H, 5, 16, 4, row0=3, stride=7, shadow=True)
    rows = list(range(3, H, 7))
    assert np.array_equal(sh["rgb"], full["rgb"].reshape(H, W, 3)[rows].reshape(-1, 3))


@pytest.mark.parametrize("model,spp,bounces,shadow", [("stanford-bunny.obj", 16, 4, "bin"),
                                                      ("suzanne.obj", 3, 3, "bin"), ("suzanne.obj", 3, 3, "lane"),
                                                      ("stanford-bunny.obj", 16, 4, "lane"),
                                                      ("teapot.obj", 4, 3, "rec"), ("teapot.obj", 4, 3, "bin"),
                                                      ("teapot.obj", 4, 2, None), ("stanford-bunny.obj", 1, 0, None)])
def test_paths_queue_matches_megakernel_and_oracle(oracle, model, spp, bounces, shadow, monkeypatch):
    """The queued pipeline (RT_PATHS=queue, queue_paths.h: the primary segments
    by the wave walk, then per bounce one compacted queue of every path's rays,
    a fall-back list for the exact per-lane traversal, and the pixel sums)
    renders the same bits as the megakernel and the oracle: packed (spp 16, 4)
    and one-sample (spp 3, 1) primary tiles, occlusion rays (RT_SHADOW_RAYS=
    bin, the default: queued, sorted by direction from the light and walked by
    the wave-cooperative any-hit walk; lane: per lane in the segment kernel;
    rec: from queued records, per lane), a strided shard, and the counts of
    segments and occlusion rays.  Packed spp 16 and 4 take the packet kernel's
    primaries and the 8-way partitioned queues."""
    if shadow:
        monkeypatch.setenv("RT_SHADOW_RAYS", shadow)
    shadow = shadow is not None
    tris = golden_scene(model)
    s = scene(model, "bsah", 8)
    pos, d = rt.CameraPath(rt.scene_center(tris), 36).circular_path(13)
    W, H = 61, 37
    monkeypatch.setenv("RT_PATHS", "mega")
    mega = _paths_render(s, pos, d, W, H, 13, spp, bounces, shadow=shadow, stats=True)
    mega_sh = _paths_render(s, pos, d, W, H, 13, spp, bounces, row0=2, stride=3, shadow=shadow)
    monkeypatch.setenv("RT_PATHS", "queue")
    q = _paths_render(s, pos, d, W, H, 13, spp, bounces, shadow=shadow, stats=True)
    q_sh = _paths_render(s, pos, d, W, H, 13, spp, bounces, row0=2, stride=3, shadow=shadow)
    for k in ("id", "dist", "rgb", "hits"):
        assert np.array_equal(q[k], mega[k]), k
        assert np.array_equal(q_sh[k], mega_sh[k]), k
    for k in ("rays", "shadow_rays", "shadow_occluded"):
        assert q["stats"][k] == mega["stats"][k], k
    o = oracle.bvh(tris, "bsah", 8).render_paths(pos, d, W, H, 13, spp, bounces, shadow=shadow)
    assert np.array_equal(q["rgb"], o["rgb"])
    assert q["rgb"].max() > 0


def test_errors_fail_loudly():
    with pytest.raises(rt.RTError, match="Unknown algorithm"):
        rt.Scene(golden_scene("teapot.obj"), "quick", 2)
    with pytest.raises(rt.RTError, match="Unsupported bvh degree"):
        rt.Scene(golden_scene("teapot.obj"), "bsah", 3)
    with pytest.raises(rt.RTError, match="invalid split position"):
        rt.Scene(np.tile(golden_scene("teapot.obj")[:1], (3, 1)), "bsah", 2)
    s = rt.Scene(golden_scene("teapot.obj"), "bsah", 2)
    with pytest.raises(rt.RTError, match="not uploaded"):
        s.calculate_screen([0, 0, 5], [0, 0, -1], 8, 8)


@pytest.mark.parametrize("shards", [1, 2, 3, 8])
def test_sharded_frames_through_the_abi_equal_one_device(monkeypatch, shards):
    """rt_render_batch_multi / rt_render_frame shard image rows over the uploaded
    devices, gather the shards to the first device and de-interleave them there
    (RCCL between distinct devices).  RT_VIRTUAL_SHARDS runs the same shard,
    gather-layout, de-interleave and hit-count code on one device (device copies
    in place of RCCL): outputs equal the unsharded render bit for bit."""
    torch = pytest.importorskip("torch")
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (0, 5, 11, 23, 30)]
    W, H, F = 203, 117, 5
    ref = {}
    for key, dt, per in (("id", torch.int32, 1), ("dist", torch.float64, 1), ("pos", torch.float64, 3),
                         ("rgb", torch.uint8, 3)):
        ref[key] = torch.empty(F * H * W * per, dtype=dt, device="cuda:0")
    ref_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ref["id"].data_ptr(), dist=ref["dist"].data_ptr(),
                          hit_pos=ref["pos"].data_ptr(), rgb=ref["rgb"].data_ptr(), hit_count=ref_cnt.data_ptr(),
                          stream=st)
    monkeypatch.setenv("RT_VIRTUAL_SHARDS", str(shards))
    got = {k: torch.full_like(v, 7) for k, v in ref.items()}
    cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_multi(cams, W, H, hit_id=got["id"].data_ptr(), dist=got["dist"].data_ptr(),
                         hit_pos=got["pos"].data_ptr(), rgb=got["rgb"].data_ptr(), hit_count=cnt.data_ptr(), stream=st)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(got[k], ref[k]), (shards, k)
    assert torch.equal(cnt, ref_cnt)
    # the blocking host-buffer frame call takes the same path
    p, d = cams[2]
    g = s.calculate_screen(p, d, W, H)
    assert np.array_equal(g["hit_id"], ref["id"].cpu().numpy().view(np.uint32).reshape(F, -1)[2])
    assert np.array_equal(g["rgb"].reshape(-1), ref["rgb"].cpu().numpy().reshape(F, -1)[2])
    assert g["hits"] == int(ref_cnt[2])
    # 4 spp (config c4's multi-GPU case): per-sample outputs, averaged colours
    # and sample hit counts through the same shards
    monkeypatch.delenv("RT_VIRTUAL_SHARDS")
    r4 = {"id": torch.empty(F * H * W * 4, dtype=torch.int32, device="cuda:0"),
          "rgb": torch.empty(F * H * W * 3, dtype=torch.uint8, device="cuda:0")}
    c4 = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=r4["id"].data_ptr(), rgb=r4["rgb"].data_ptr(),
                          hit_count=c4.data_ptr(), stream=st, spp=4)
    monkeypatch.setenv("RT_VIRTUAL_SHARDS", str(shards))
    g4 = {k: torch.full_like(v, 7) for k, v in r4.items()}
    g4c = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_multi(cams, W, H, hit_id=g4["id"].data_ptr(), rgb=g4["rgb"].data_ptr(), hit_count=g4c.data_ptr(),
                         stream=st, spp=4)
    torch.cuda.synchronize()
    for k in r4:
        assert torch.equal(g4[k], r4[k]), (shards, "spp4", k)
    assert torch.equal(g4c, c4)


@pytest.mark.parametrize("spp", [1, 4])
def test_rccl_group_branch_equals_one_device(monkeypatch, spp):
    """The RCCL branch of render_group (rt_api.cpp): RT_GROUP_RCCL=1 sends a
    one-device scene through the multi-device path with its real transport — a
    one-rank communicator from ncclCommInitAll over {0}, created lazily on the
    first group render; ncclGroupStart / ncclGather / ncclGroupEnd of the
    staging block into the root buffer; k_deinterleave / k_sum_counts — through
    rt_render_batch_multi and rt_render_frame.  Outputs equal the one-device
    render bit for bit (the multi-GPU drop-in path, INTEGRATION.md §2,
    replacing src/main.cpp:253-255)."""
    torch = pytest.importorskip("torch")
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (1, 8, 27)]
    W, H, F = 211, 97, 3
    st = torch.cuda.current_stream().cuda_stream
    want = (("id", torch.int32, spp), ("dist", torch.float64, spp), ("pos", torch.float64, 3 * spp),
            ("rgb", torch.uint8, 3))
    ref = {k: torch.empty(F * H * W * per, dtype=dt, device="cuda:0") for k, dt, per in want}
    ref_cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
    s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=ref["id"].data_ptr(), dist=ref["dist"].data_ptr(),
                          hit_pos=ref["pos"].data_ptr(), rgb=ref["rgb"].data_ptr(), hit_count=ref_cnt.data_ptr(),
                          stream=st, spp=spp)
    monkeypatch.setenv("RT_GROUP_RCCL", "1")
    for it in range(2):  # the second call reuses the communicator and the staging blocks
        got = {k: torch.full_like(v, 7) for k, v in ref.items()}
        cnt = torch.zeros(F, dtype=torch.int64, device="cuda:0")
        s.render_batch_multi(cams, W, H, hit_id=got["id"].data_ptr(), dist=got["dist"].data_ptr(),
                             hit_pos=got["pos"].data_ptr(), rgb=got["rgb"].data_ptr(), hit_count=cnt.data_ptr(),
                             stream=st, spp=spp)
        torch.cuda.synchronize()
        for k in ref:
            assert torch.equal(got[k], ref[k]), (spp, it, k)
        assert torch.equal(cnt, ref_cnt), (spp, it)
    if spp == 1:
        # the blocking host-buffer frame call (rt_render_frame) over the group
        p, d = cams[1]
        g = s.calculate_screen(p, d, W, H, want=("hit_id", "dist", "rgb"))
        assert np.array_equal(g["hit_id"], ref["id"].cpu().numpy().view(np.uint32).reshape(F, -1)[1])
        assert np.array_equal(g["dist"], ref["dist"].cpu().numpy().reshape(F, -1)[1])
        assert np.array_equal(g["rgb"].reshape(-1), ref["rgb"].cpu().numpy().reshape(F, -1)[1])
        assert g["hits"] == int(ref_cnt[1])


def test_band_shards_reassemble_to_full_frame():
    """rt_render_shard_device (bands of 8 rows interleaved over the shards, the
    multi-GPU partition bench.py uses) reassembles through shards.py into the
    one-device frame bit for bit, for even and uneven shard counts."""
    torch = pytest.importorskip("torch")
    from raytracingdemo_amd.shards import deinterleave_into, rows_per_rank
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in (2, 19)]
    W, H, F = 150, 101, 2
    full = [s.calculate_screen(p, d, W, H) for p, d in cams]
    st = torch.cuda.current_stream().cuda_stream
    for G in (1, 2, 3, 8):
        R = rows_per_rank(H, G)
        ids = torch.full((G, F, R, W), -7, dtype=torch.int32, device="cuda:0")
        rgb = torch.zeros((G, F, R, W, 3), dtype=torch.uint8, device="cuda:0")
        cnt = torch.zeros((G, F), dtype=torch.int64, device="cuda:0")
        for g in range(G):
            n = rt.shard_height(H, G, g)
            t_id = torch.empty((F, n, W), dtype=torch.int32, device="cuda:0")
            t_rgb = torch.empty((F, n, W, 3), dtype=torch.uint8, device="cuda:0")
            s.render_shard_device(0, cams, W, H, g, G, hit_id=t_id.data_ptr(), rgb=t_rgb.data_ptr(),
                                  hit_count=cnt[g].data_ptr(), stream=st)
            ids[g, :, :n] = t_id
            rgb[g, :, :n] = t_rgb
        torch.cuda.synchronize()
        img_id = deinterleave_into(ids, H, torch.empty((F, H, W), dtype=torch.int32, device="cuda:0"))
        img_rgb = deinterleave_into(rgb, H, torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda:0"))
        for f in range(F):
            assert np.array_equal(img_id[f].cpu().numpy().view(np.uint32).reshape(-1), full[f]["hit_id"]), (G, f)
            assert np.array_equal(img_rgb[f].cpu().numpy().reshape(-1, 3), full[f]["rgb"]), (G, f)
            assert int(cnt[:, f].sum()) == full[f]["hits"], (G, f)


def test_concurrent_callers_on_one_scene():
    """Two host threads drive one scene at once (rt_render_frame, blocking,
    and rt_render_batch_device on their own streams; ctypes drops the GIL in
    the calls): the library serialises them on the scene's lock and every
    result equals the sequential one (include/rt.h threading note)."""
    import threading

    torch = pytest.importorskip("torch")
    tris = golden_scene("stanford-bunny.obj")
    s = scene("stanford-bunny.obj", "bsah", 8)
    path = rt.CameraPath(rt.scene_center(tris), 36)
    cams = [path.circular_path(f) for f in range(12)]
    W, H = 200, 120
    ref = [s.calculate_screen(p, d, W, H, want=("hit_id", "rgb")) for p, d in cams]
    errors: list = []

    def frames(k):
        try:
            out = None
            for it in range(3):
                for f in range(k, len(cams), 2):
                    out = s.calculate_screen(*cams[f], W, H, want=("hit_id", "rgb"), out=out)
                    assert np.array_equal(out["hit_id"], ref[f]["hit_id"]), (k, it, f)
                    assert np.array_equal(out["rgb"], ref[f]["rgb"]), (k, it, f)
        except BaseException as e:  # reported by the main thread
            errors.append(e)

    def batches():
        try:
            st = torch.cuda.Stream()
            t_id = torch.empty(len(cams) * W * H, dtype=torch.int32, device="cuda:0")
            for it in range(3):
                s.render_batch_device(0, cams, W, H, 0, 1, H, hit_id=t_id.data_ptr(), stream=st.cuda_stream)
                st.synchronize()
                got = t_id.cpu().numpy().view(np.uint32).reshape(len(cams), -1)
                for f in range(len(cams)):
                    assert np.array_equal(got[f], ref[f]["hit_id"]), ("batch", it, f)
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=frames, args=(0,)), threading.Thread(target=frames, args=(1,)),
          threading.Thread(target=batches)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a caller thread hung"
    if errors:
        raise errors[0]
