"""The C ABI library (CPU-only checks: no compute call needs a GPU here).

librtmi355x.so loads, exports every function include/rt.h declares, reports
the header's ABI version, and its host-only entry points (loader, scene build,
camera path, tree dump) work without a device.  Device entry points must fail
loudly (RT_ERR_NO_DEVICE) rather than fall back to the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rt.h")


def _lib():
    from raytracingdemo_amd import _native as N
    if not os.path.exists(N.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracingdemo_amd", "csrc")], check=True)
    return N, N.lib()


def declared_functions() -> list[str]:
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rt_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "rt_render_frame" in names and "rt_scene_create" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    N, L = _lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(N.EXPORTS) == declared_functions()


def test_abi_version_matches_header():
    _, L = _lib()
    v = int(re.search(r"#define RT_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert L.rt_abi_version() == v


def test_status_codes_match_header():
    N, _ = _lib()
    src = open(HEADER).read()
    for name in ("RT_OK", "RT_ERR_INVALID_ARGUMENT", "RT_ERR_OUT_OF_RANGE", "RT_ERR_RUNTIME", "RT_ERR_HIP",
                 "RT_ERR_NO_DEVICE", "RT_MODE_EXACT", "RT_MODE_FP64", "RT_FLAG_COUNT", "RT_FLAG_TIMING",
                 "RT_FLAG_SHADOW", "RT_FLAG_SIDE_SLOT", "RT_FLAG_COUNTS_STORE"):
        v = int(re.search(rf"#define {name} (\d+)", src).group(1))
        assert getattr(N, name) == v, name


def test_frame_stats_struct_matches_header():
    """The ctypes mirror has exactly the header's rt_frame_stats_t fields, in order."""
    N, _ = _lib()
    src = open(HEADER).read()
    end = src.index("} rt_frame_stats_t;")
    body = src[src.rindex("typedef struct {", 0, end) + len("typedef struct {"):end]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        for name in decl.split(None, 1)[1].split(","):
            fields.append(re.sub(r"\[.*\]", "", name).strip())
    assert [f for f, _ in N.rt_frame_stats_t._fields_] == fields


def test_last_error_is_a_string():
    _, L = _lib()
    assert isinstance(L.rt_last_error(), bytes)


def test_device_calls_fail_loudly_without_upload():
    """No CPU fallback: rendering a scene that is on no device is an error."""
    import numpy as np
    import raytracingdemo_amd as rt
    tri = np.array([[-1.0, -1.0, 0.0, 1.0, -1.0, 0.0, 0.0, 1.0, 0.0]])
    s = rt.Scene(tri, "bsah", 2)
    with pytest.raises(rt.RTError, match="not uploaded"):
        s.calculate_screen([0, 0, 5], [0, 0, -1], 8, 8)


def test_batch_render_rejects_mixed_sizes_and_needs_a_device():
    """rt_render_batch_device: every pose of a batch shares one image size, and
    without an uploaded replica the call fails loudly (no CPU fallback)."""
    N, L = _lib()
    import numpy as np
    import raytracingdemo_amd as rt
    from conftest import golden_scene
    s = rt.Scene(golden_scene("teapot.obj"), "bsah", 4)
    cams = (N.rt_camera * 2)(rt._camera([0, 0, 5], [0, 0, -1], 8, 8), rt._camera([0, 0, 5], [0, 0, -1], 8, 6))
    o = N.rt_device_out()
    st = L.rt_render_batch_device(s.handle, 0, cams, 2, N.RT_MODE_EXACT, 0, 1, 6, C.byref(o), None, 0)
    assert st == N.RT_ERR_INVALID_ARGUMENT
    assert b"share the image size" in L.rt_last_error()
    cams[1].height = 8
    st = L.rt_render_batch_device(s.handle, 0, cams, 2, N.RT_MODE_EXACT, 0, 1, 8, C.byref(o), None, 0)
    assert st != N.RT_OK
    assert L.rt_render_batch_device(s.handle, 0, cams, -1, N.RT_MODE_EXACT, 0, 1, 8, C.byref(o), None, 0) \
        == N.RT_ERR_INVALID_ARGUMENT
    assert np.isfinite(s.tris).all()


def test_shard_render_job_is_validated_before_any_device_work():
    """rt_render_shard_device_job rejects a malformed de-interleave job
    (no shards, no buffers, frame_rows below a shard's rows) with
    RT_ERR_INVALID_ARGUMENT, and a well-formed one still needs an uploaded
    replica (no CPU fallback)."""
    N, L = _lib()
    import numpy as np
    import raytracingdemo_amd as rt
    from conftest import golden_scene
    s = rt.Scene(golden_scene("teapot.obj"), "bsah", 8)
    cams = (N.rt_camera * 1)(rt._camera([0, 0, 5], [0, 0, -1], 16, 16))
    o = N.rt_device_out()
    buf = np.zeros(4096, dtype=np.uint8)
    good = dict(gathered=buf.ctypes.data, block_bytes=1024, section_offset=0, shards=2, frames=1, height=16,
                width=16, elem_bytes=3, frame_rows=8, frames_out=buf.ctypes.data)
    for bad in (dict(shards=0), dict(gathered=None), dict(frames_out=None), dict(frame_rows=4), dict(elem_bytes=0),
                dict(block_bytes=8 * 16 * 3 - 1), dict(section_offset=1024 - 8 * 16 * 3 + 1),
                dict(frame_rows=0, block_bytes=8 * 16 * 3 - 1)):
        j = N.rt_deinterleave_job(**{**good, **bad})
        st = L.rt_render_shard_device_job(s.handle, 0, cams, 1, 1, N.RT_MODE_EXACT, 0, 2, C.byref(o), C.byref(j),
                                          None, 0)
        assert st == N.RT_ERR_INVALID_ARGUMENT, bad
        assert b"de-interleave job" in L.rt_last_error()
    j = N.rt_deinterleave_job(**good)
    st = L.rt_render_shard_device_job(s.handle, 0, cams, 1, 1, N.RT_MODE_EXACT, 0, 2, C.byref(o), C.byref(j), None, 0)
    assert st != N.RT_OK and b"not uploaded" in L.rt_last_error()


def test_upload_rejects_repeated_or_negative_device_ordinals():
    """rt_scene_upload's device list is the rank order of the RCCL communicator
    a multi-device render creates (ncclCommInitAll): a
    negative or repeated ordinal is RT_ERR_INVALID_ARGUMENT before any device
    or RCCL call (so here too, without a GPU); an ordinal past the device
    count is RT_ERR_INVALID_ARGUMENT on a GPU box, RT_ERR_NO_DEVICE here."""
    N, L = _lib()
    import raytracingdemo_amd as rt
    from conftest import golden_scene
    s = rt.Scene(golden_scene("teapot.obj"), "bsah", 8)
    for devs, msg in (([0, 0], b"listed twice"), ([1, 0, 1], b"listed twice"), ([-1], b"negative")):
        arr = (C.c_int * len(devs))(*devs)
        assert L.rt_scene_upload(s.handle, arr, len(devs)) == N.RT_ERR_INVALID_ARGUMENT, devs
        assert msg in L.rt_last_error(), devs
    assert L.rt_scene_upload(s.handle, None, -1) == N.RT_ERR_INVALID_ARGUMENT
    arr = (C.c_int * 1)(4096)
    assert L.rt_scene_upload(s.handle, arr, 1) in (N.RT_ERR_INVALID_ARGUMENT, N.RT_ERR_NO_DEVICE)


@pytest.mark.parametrize("G,F,H,W,eb", [(1, 2, 5, 3, 4), (2, 3, 7, 5, 3), (3, 2, 1080, 16, 8), (8, 1, 1081, 9, 24),
                                        (5, 4, 3, 2, 1)])
def test_deinterleave_rows_matches_row_interleaving(G, F, H, W, eb):
    """rt_deinterleave_rows (the host twin of the device kernel that
    rt_render_batch_multi runs after the RCCL gather): shard g holds the bands
    of 8 image rows b = g, g + G, ... of every frame; the de-interleave puts
    row j of frame f back from shard (j // 8) % G (each shard's frames back to
    back in its block, as its shard render wrote them)."""
    import numpy as np
    import raytracingdemo_amd as rt
    rng = np.random.default_rng(G * 1000 + H)
    frames = rng.integers(0, 256, size=(F, H, W * eb), dtype=np.uint8)
    R = -(-(-(-H // 8)) // G) * 8  # rows of the tallest shard
    sec_off, pad = 256, 64  # a section inside each block, as the library lays it out
    block = sec_off + F * R * W * eb + pad  # sized for the tallest shard
    gathered = rng.integers(0, 256, size=(G, block), dtype=np.uint8)  # the unused tail stays garbage
    from raytracingdemo_amd.shards import shard_rows
    for g in range(G):
        mine = shard_rows(g, G, H)  # bands of 8 rows, band b on shard b % G
        assert len(mine) == rt.shard_height(H, G, g)
        rows = np.ascontiguousarray(frames[:, mine]).reshape(-1)  # [F, rows_g, W*eb], frames back to back
        gathered[g, sec_off:sec_off + len(rows)] = rows
    out = rt.deinterleave_rows(gathered, G, F, H, W, eb, block_bytes=block, section_offset=sec_off)
    assert np.array_equal(out, frames)
