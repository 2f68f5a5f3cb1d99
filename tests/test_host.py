"""The product's host-side stages against the reference (CPU only, no GPU).

The library builds the reference's own tree on the host (src/stack_bvh.hpp
build/partition/collapse), loads OBJs with objl's semantics (lib/OBJ_Loader.h)
and walks the reference's camera path (src/camera_path.hpp).  These are pinned
here against the reference's tree digests (tests/golden/ref_trees.json: 21
algorithms x 3 models), the published camera strings and the oracle loader.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import raytracingdemo_amd as rt
from conftest import golden_scene

MODELS = ["teapot.obj", "suzanne.obj", "stanford-bunny.obj"]


def _digest(t) -> str:
    h = hashlib.sha256()
    for a in (t.boxes, t.meta, t.order):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("model", MODELS)
def test_product_trees_match_reference(trees_golden, model):
    """rt_scene_create builds the reference's exact tree for every algorithm."""
    tris = golden_scene(model)
    for name, exp in trees_golden[model]["trees"].items():
        algo, k = name.rsplit("-", 1)
        t = rt.Scene(tris, algo, int(k)).tree_dump()
        assert len(t.meta) == exp["nodes"], name
        assert _digest(t) == exp["sha256"], name


def test_product_camera_path_matches_published_csv(frames_golden):
    for model in MODELS:
        tris = golden_scene(model)
        path = rt.CameraPath(rt.scene_center(tris), 36)
        for f in frames_golden[model]["frames"]:
            pos, d = path.circular_path(f["step"])
            assert ["%g" % x for x in pos] == f["cam_pos"]
            assert ["%g" % x for x in d] == f["cam_dir"]


def test_product_scene_center_matches_oracle(oracle):
    for model in MODELS:
        tris = golden_scene(model)
        assert np.array_equal(rt.scene_center(tris), oracle.scene_center(tris))


OBJ_TEXT = """# objl corner cases: n-gons (ear clipping), negative/relative indices,
# texture/normal slots, groups and materials splitting meshes
o first
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 1.5 0
vt 0 0
vn 0 0 1
f 1/1/1 2/1/1 3/1/1 4/1/1 5/1/1
g second
usemtl red
v 2 0 0
v 3 0 0
v 3 1 0
f -3 -2 -1
v 4 0 1.25
v 5 0 1.5
v 5 2 1.75
v 4 2 2
f 9//1 10//1 11//1 12//1
"""


def test_product_loader_matches_oracle_loader(oracle, tmp_path):
    p = tmp_path / "corner.obj"
    p.write_text(OBJ_TEXT)
    for scale in (1.0, 0.035, 30.0):
        a = rt.ObjectLoader.load_from_file(str(p), scale)
        b = oracle.load_obj(str(p), scale)
        assert a.shape == b.shape and a.shape[0] >= 5
        assert np.array_equal(a, b)


def test_product_loader_missing_file():
    with pytest.raises(rt.RTError, match="Failed to load OBJ file"):
        rt.ObjectLoader.load_from_file("/nonexistent/none.obj")


def test_product_errors_match_reference():
    tris = golden_scene("teapot.obj")
    with pytest.raises(rt.RTError, match="Unknown algorithm"):
        rt.Scene(tris, "quick", 2)
    with pytest.raises(rt.RTError, match="Unsupported bvh degree"):
        rt.Scene(tris, "bsah", 3)
    with pytest.raises(rt.RTError, match="invalid split position"):
        rt.Scene(np.tile(tris[:1], (3, 1)), "bsah", 2)


def test_scene_triangle_cap():
    """Scenes above RT_MAX_TRIS (the packet walk's 32-bit record offsets) are
    refused before the triangle array is read (a 1-triangle buffer with a
    larger count is never touched)."""
    import ctypes as C
    from raytracingdemo_amd import _native as N
    one = np.zeros(9, dtype=np.float64)
    h = C.c_void_p()
    st = N.lib().rt_scene_create(one.ctypes.data, 83_886_081, 0, 8, 0, C.byref(h))
    assert st == 1 and not h.value  # RT_ERR_INVALID_ARGUMENT
    assert "too many triangles" in N.lib().rt_last_error().decode()


def test_threaded_tree_build_equals_the_serial_loop(monkeypatch):
    """build_tree hands large subtrees to threads and splices them back into
    the reference's node numbering (csrc/bvh_build.cpp grow_parallel); on the
    headline scene (262,267 triangles: three threaded levels for the 2-way
    variants) it equals the reference's serial work-stack loop node for node.
    The bunny goldens above pin the threaded build to the reference itself.
    The flatten that follows (per-triangle records on threads, the walk
    tree's top subtrees filled apart and spliced) must produce the same
    device scene byte for byte (rt_scene_stats layout_digest)."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    for algo, k in [("bsah", 8), ("sah-c", 8), ("median", 2)]:
        monkeypatch.setenv("RT_BUILD_THREADS", "1")
        a = rt.Scene(tris, algo, k)
        serial, serial_layout = _digest(a.tree_dump()), a.stats()["layout_digest"]
        del a
        monkeypatch.delenv("RT_BUILD_THREADS")
        b = rt.Scene(tris, algo, k)
        assert _digest(b.tree_dump()) == serial, (algo, k)
        assert b.stats()["layout_digest"] == serial_layout, (algo, k)


def test_threaded_tree_build_reports_a_subtree_error():
    """A split error inside a threaded subtree comes back as the reference's
    exception ("invalid split position" on duplicate triangles), not a crash."""
    tris = golden_scene("stanford-bunny.obj")
    with pytest.raises(rt.RTError, match="invalid split position"):
        rt.Scene(np.concatenate([tris, tris]), "bsah", 2)


def test_scene_stats_are_consistent():
    tris = golden_scene("stanford-bunny.obj")
    for algo, k in [("bsah", 2), ("bsah", 8), ("sah-c", 16), ("median", 4)]:
        st = rt.Scene(tris, algo, k).stats()
        assert st["triangles"] == len(tris)
        assert st["real_nodes"] == st["real_inner"] + st["real_leaves"]
        if st["walk_tree"]:  # rebuilt SAH walk tree: always 8-wide
            assert st["wide_width"] == 8
        else:
            assert st["wide_width"] in (2, 4, 8, 16) and st["wide_width"] >= min(k, 16)
        assert st["node_bytes"] == 32 * st["wide_width"]
        assert 1 <= st["stack_bound"] <= st["depth"] * (st["wide_width"] - 1) + 1 + st["depth"] * 16


def test_scene_cache_returns_the_loader_output(tmp_path):
    """rt_load_obj_cached: a miss parses and writes the entry, a hit returns the
    loader's triangles bit for bit; an edited OBJ or a corrupted entry is parsed
    again."""
    from raytracingdemo_amd.scenes import write_obj
    tris = golden_scene("teapot.obj")
    obj = tmp_path / "teapot.obj"
    write_obj(tris, str(obj))
    cache = tmp_path / "cache"
    direct = rt.load_obj(str(obj), 2.5)
    a, hit_a = rt.load_obj_cached(str(obj), 2.5, str(cache))
    b, hit_b = rt.load_obj_cached(str(obj), 2.5, str(cache))
    assert (hit_a, hit_b) == (False, True)
    assert np.array_equal(a, direct) and np.array_equal(b, direct)
    c, hit_c = rt.load_obj_cached(str(obj), 1.0, str(cache))  # another scale: another key
    assert not hit_c and np.array_equal(c, rt.load_obj(str(obj), 1.0))
    entries = sorted(cache.glob("*.rtsc"))
    assert len(entries) == 1  # same OBJ bytes: one digest, the entry now holds scale 1.0
    raw = bytearray(entries[0].read_bytes())
    raw[-1] ^= 0xFF  # corrupt the payload
    entries[0].write_bytes(bytes(raw))
    d, hit_d = rt.load_obj_cached(str(obj), 1.0, str(cache))
    assert not hit_d and np.array_equal(d, c)
    with open(obj, "a") as fh:
        fh.write("v 1 2 3\nv 2 3 4\nv 3 4 6\nf -3 -2 -1\n")
    e, hit_e = rt.load_obj_cached(str(obj), 1.0, str(cache))
    assert not hit_e and len(e) == len(c) + 1
    with pytest.raises(rt.RTError, match="Failed to load OBJ file"):
        rt.load_obj_cached(str(tmp_path / "missing.obj"), 1.0, str(cache))


def test_calculate_screen_rejects_mismatched_output_arrays():
    """calculate_screen(out=...) reuses the caller's host arrays (runTest's
    reused ray_hits); a wrong shape or dtype is refused before any device call."""
    s = rt.Scene(golden_scene("teapot.obj"), "bsah", 2)
    W, H = 16, 8
    ok = {"hit_id": np.empty(W * H, np.uint32), "dist": np.empty(W * H), "pos": None,
          "rgb": np.empty((W * H, 3), np.uint8)}
    for key, bad in [("hit_id", np.empty(W * H, np.int64)), ("dist", np.empty(W * H + 1)),
                     ("rgb", np.empty((W * H, 3), np.uint8)[:, ::-1])]:
        out = dict(ok)
        out[key] = bad
        with pytest.raises(ValueError, match=key):
            s.calculate_screen([0, 0, 5], [0, 0, -1], W, H, out=out)


def test_planned_collapse_is_deterministic_and_smaller(monkeypatch):
    """The SAH-optimal 8-wide collapse of the walk tree (walk_tree.cpp
    plan_wide_collapse) is a pure function of the binary tree: two builds give
    the same device layout, and it needs fewer wide nodes than the greedy
    collapse (RT_WALK_COLLAPSE=greedy) on the headline scene."""
    from raytracingdemo_amd.scenes import sponza_proxy_triangles
    tris = sponza_proxy_triangles()
    a = rt.Scene(tris, "bsah", 8).stats()
    b = rt.Scene(tris, "bsah", 8).stats()
    assert a["walk_tree"] == 1 and a["layout_digest"] == b["layout_digest"]
    monkeypatch.setenv("RT_WALK_COLLAPSE", "greedy")
    g = rt.Scene(tris, "bsah", 8).stats()
    assert g["layout_digest"] != a["layout_digest"]
    assert a["wide_nodes"] < 0.7 * g["wide_nodes"], (a["wide_nodes"], g["wide_nodes"])
    assert a["triangles"] == g["triangles"] and a["max_leaf_size"] <= 16


def test_pmc_traffic_sums_the_queued_pipeline_per_pose(tmp_path):
    """tools/pmc_traffic.py "queue": the queued path tracer's kernels summed per
    pose, the counting pose (COUNT instantiations and everything before the
    first timed k_q_primary) left out; pmc_valu.py reads the same sums."""
    import csv
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import pmc_traffic
    rows = []
    names = ["k_q_primary<8, 1, true, true, true>(", "k_q_segment<8, 8, 4, true, 1>(", "k_q_accum(",  # counting pose
             "k_q_primary<8, 1, false, true, true>(", "k_q_segment<8, 8, 4, false, 1>(", "k_sh_scatter(", "k_q_accum(",
             "k_trace_packet<8, 128, 8, false, true, false, false>(",  # not the pipeline's
             "k_q_primary<8, 1, false, true, true>(", "k_q_segment<8, 8, 4, false, 1>(", "k_q_accum(",
             # packet-kernel primaries: the counting one skipped, the timed one starts a pose
             "k_trace_packet<8, 128, 8, true, true, true, false, true>(",
             "k_trace_packet<8, 128, 8, false, true, true, false, true>(", "k_q_segment<8, 8, 5, false, 2>(",
             "k_sh_walk<8, false>("]
    for d, n in enumerate(names):
        rows.append({"Dispatch_Id": str(d + 1), "Kernel_Name": "void (anonymous namespace)::" + n + "RtDevScene)",
                     "Counter_Name": "FETCH_SIZE", "Counter_Value": str(10.0 * (d + 1))})
    path = tmp_path / "f.csv"
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    poses = pmc_traffic.per_pose(str(path))
    assert sorted(poses) == [0, 1, 2]
    assert poses[0]["FETCH_SIZE"] == 40 + 50 + 60 + 70
    assert poses[1]["FETCH_SIZE"] == 90 + 100 + 110
    assert poses[2]["FETCH_SIZE"] == 130 + 140 + 150
    assert pmc_traffic.queue_counting("k_sh_lane<8, 8, true>(") and not pmc_traffic.queue_counting("k_sh_lane<8, 8, false>(")


# One process, one RCCL, and a clean exit in either import order.  Round 4
# found "double free or corruption (!prev)" at exit after torch's librccl.so
# had been mapped RTLD_GLOBAL ahead of `import torch` (fixed in _native.py);
# the library now reuses the RCCL the process holds and opens ROCm's
# RTLD_LOCAL only when none is mapped (rt_api.cpp rccl()).
_CHILD = r"""
import sys
sys.path.insert(0, {root!r})
order = {order!r}
if order == "torch_first":
    import torch
    import raytracingdemo_amd as rt
    rt._native.lib()
else:
    import raytracingdemo_amd as rt
    rt._native.lib()
    import torch
    # the multi-device upload path's own step: torch's RCCL first
    rt._native.prefer_torch_rccl()
L = rt._native.lib()
p = L.rt_rccl_path()
assert p, L.rt_last_error()
maps = {{ln.split()[-1] for ln in open("/proc/self/maps") if "librccl" in ln}}
print("RCCL", p.decode(), "MAPPED", sorted(maps))
"""


@pytest.mark.parametrize("order", ["torch_first", "library_first"])
def test_import_orders_exit_cleanly_with_one_rccl(order):
    import os
    import subprocess
    import sys

    torch = pytest.importorskip("torch")
    if not os.path.exists(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")):
        pytest.skip("this PyTorch ships no RCCL")

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=root, order=order)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "double free" not in r.stderr and "corruption" not in r.stderr, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RCCL ")][-1]
    path, mapped = line[5:].split(" MAPPED ")
    mapped = eval(mapped)  # a list literal printed by the child
    assert len(mapped) == 1, mapped           # never two copies
    torch_rccl = os.path.realpath(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
    assert os.path.realpath(path) == torch_rccl  # the process's (PyTorch's) copy


def test_tile_division_magic():
    """packet_kernel.h div_magic / div_by (the per-tile division by the tiles
    per frame and per tile row): the multiply-high form equals integer
    division for every n < 2^31, here over divisors 1..4096, large and
    power-of-two ones, and the n that stress each (multiples, their
    neighbours, 2^31 - 1)."""
    import random

    def magic(d):  # the device code's arithmetic, step for step
        l = (d - 1).bit_length() if d > 1 else 0
        P = 1 << (31 + l)
        q = min(int(float(P) / float(d)), 0xFFFFFFFF)
        while q * d < P:
            q += 1
        while q > 1 and (q - 1) * d >= P:
            q -= 1
        assert q < 1 << 32
        return q, 31 + l

    rng = random.Random(7)
    ds = list(range(1, 4097)) + [240 * 135, 480 * 270, 32400 * 36, (1 << 31) - 1, 1 << 30, 3 << 29]
    ds += [rng.randrange(1, 1 << 31) for _ in range(200)]
    for d in ds:
        m, sh = magic(d)
        ns = [0, 1, d - 1, d, d + 1, (1 << 31) - 1, ((1 << 31) - 1) // d * d, ((1 << 31) - 1) // d * d - 1]
        ns += [rng.randrange(0, 1 << 31) for _ in range(20)]
        for n in ns:
            if 0 <= n < 1 << 31:
                assert (n * m) >> sh == n // d, (d, n)
