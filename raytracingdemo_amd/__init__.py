"""raytracingdemo_amd — MI355X-native primary-ray tracer (host-side mirror).

Python view of the C ABI in include/rt.h, named after the reference's own
objects so tests and drivers read like the reference:

    ObjectLoader.load_from_file  ~ ObjectLoader::loadFromFile (src/utils/object_loader.hpp:14)
    scene_center                 ~ runTest's centre (src/main.cpp:118-122)
    CameraPath.circular_path     ~ CameraPath::circularPath (src/camera_path.hpp:18)
    Scene(tris, algorithm, k)    ~ StackBVH::build (+collapse)  (src/stack_bvh.hpp:502,574)
    Scene.calculate_screen       ~ calculateScreen + shadeScreen (src/main.cpp:322-381)

Algorithm names follow the reference's runner: "bsah", "sah", "median" and the
collapsed "-c" variants (src/main.cpp:60-82, 128-205); unknown names raise the
reference's errors ("Unknown algorithm" -> out_of_range, "Unsupported bvh degree"
-> invalid_argument).  All compute runs in the gfx950 HIP kernels of
librtmi355x.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import RTError, RT_MISS

__all__ = ["RTError", "RT_MISS", "ObjectLoader", "scene_center", "CameraPath", "Scene", "ppm_bytes",
           "parse_algorithm", "load_obj"]

ALGORITHMS = {"median": 0, "sah": 1, "bsah": 2}


def parse_algorithm(name: str):
    """Runner algorithm name -> (algo id, collapse flag) (src/main.cpp:128-205)."""
    collapse = name.endswith("-c")
    base = name[:-2] if collapse else name
    if base not in ALGORITHMS:
        raise RTError(N.RT_ERR_OUT_OF_RANGE, "Unknown algorithm")
    return ALGORITHMS[base], collapse


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def load_obj(path: str, scale: float = 1.0) -> np.ndarray:
    """Triangle soup (N, 9) float64 in loader order (objl semantics)."""
    L = N.lib()
    buf = C.POINTER(C.c_double)()
    n = C.c_uint64()
    N.check(L.rt_load_obj(str(path).encode(), float(scale), C.byref(buf), C.byref(n)))
    try:
        if n.value == 0:
            return np.zeros((0, 9))
        return np.ctypeslib.as_array(buf, shape=(n.value * 9,)).copy().reshape(-1, 9)
    finally:
        L.rt_free(buf)


def load_obj_cached(path: str, scale: float = 1.0, cache_dir: str = "") -> tuple[np.ndarray, bool]:
    """load_obj through the binary scene cache (include/rt.h rt_load_obj_cached):
    (triangles, True if the cache entry was used).  cache_dir defaults to
    $RT_SCENE_CACHE or ~/.cache/rtmi355x."""
    cache_dir = cache_dir or os.environ.get("RT_SCENE_CACHE") or os.path.expanduser("~/.cache/rtmi355x")
    os.makedirs(cache_dir, exist_ok=True)
    L = N.lib()
    buf = C.POINTER(C.c_double)()
    n = C.c_uint64()
    hit = C.c_int(0)
    N.check(L.rt_load_obj_cached(str(path).encode(), float(scale), cache_dir.encode(), C.byref(buf), C.byref(n),
                                 C.byref(hit)))
    try:
        if n.value == 0:
            return np.zeros((0, 9)), bool(hit.value)
        return np.ctypeslib.as_array(buf, shape=(n.value * 9,)).copy().reshape(-1, 9), bool(hit.value)
    finally:
        L.rt_free(buf)


class ObjectLoader:
    @staticmethod
    def load_from_file(path: str, scale: float = 1.0) -> np.ndarray:
        return load_obj(path, scale)


def scene_center(tris: np.ndarray) -> np.ndarray:
    t = np.ascontiguousarray(tris, dtype=np.float64)
    out = np.zeros(3)
    N.check(N.lib().rt_scene_center(t.ctypes.data, len(t), _dp(out)))
    return out


class CameraPath:
    """Orbit of radius 5 around the scene centre (src/camera_path.hpp:18-26)."""

    def __init__(self, scene_center_xyz, resolution: int = 36):
        self.center = np.ascontiguousarray(scene_center_xyz, dtype=np.float64)
        self.resolution = int(resolution)

    def circular_path(self, step: int):
        pos, d = np.zeros(3), np.zeros(3)
        N.check(N.lib().rt_camera_path(_dp(self.center), self.resolution, int(step), _dp(pos), _dp(d)))
        return pos, d


@dataclass
class TreeDump:
    boxes: np.ndarray
    meta: np.ndarray
    order: np.ndarray


def _camera(pos, d, W, H) -> N.rt_camera:
    c = N.rt_camera()
    for a in range(3):
        c.pos[a] = float(pos[a])
        c.dir[a] = float(d[a])
    c.width, c.height = int(W), int(H)
    return c


class Scene:
    """A scene built into the reference's BVH and flattened for gfx950."""

    def __init__(self, tris: np.ndarray, algorithm: str = "bsah", k: int = 8, walk_device: int | None = None):
        """walk_device: build the walk tree on that HIP device (rt_scene_create_on_device)
        instead of the host."""
        algo, collapse = parse_algorithm(algorithm)
        self.tris = np.ascontiguousarray(tris, dtype=np.float64).reshape(-1, 9)
        self.algorithm, self.k = algorithm, int(k)
        h = C.c_void_p()
        if walk_device is None:
            N.check(N.lib().rt_scene_create(self.tris.ctypes.data, len(self.tris), algo, int(k), int(collapse),
                                            C.byref(h)))
        else:
            N.check(N.lib().rt_scene_create_on_device(self.tris.ctypes.data, len(self.tris), algo, int(k),
                                                      int(collapse), int(walk_device), C.byref(h)))
        self._h = h
        self.devices: list[int] = []

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().rt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def upload(self, devices=(0,)):
        if len(devices) > 1:
            N.prefer_torch_rccl()  # one RCCL per process (the multi-device render's gather)
        devs = (C.c_int * len(devices))(*devices)
        N.check(N.lib().rt_scene_upload(self._h, devs, len(devices)))
        self.devices = list(devices)
        return self

    def build_times(self) -> dict:
        """Stage times of the scene's creation (include/rt.h rt_scene_build_times)."""
        t = N.rt_build_times_t()
        N.check(N.lib().rt_scene_build_times(self._h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in t._fields_ if f != "reserved"}

    def stats(self) -> dict:
        s = N.rt_scene_stats_t()
        N.check(N.lib().rt_scene_stats(self._h, C.byref(s)))
        out = {}
        for f, _ in s._fields_:
            v = getattr(s, f)
            out[f] = list(v) if isinstance(v, C.Array) else v
        return out

    def tree_dump(self) -> TreeDump:
        st = self.stats()
        n = st["real_nodes"]
        boxes = np.zeros((n, 6))
        meta = np.zeros((n, 3), dtype=np.int64)
        order = np.zeros(len(self.tris), dtype=np.int64)
        N.check(N.lib().rt_scene_tree_dump(self._h, boxes.ctypes.data, meta.ctypes.data, order.ctypes.data))
        return TreeDump(boxes, meta, order)

    def calculate_screen(self, pos, d, W: int, H: int, mode: str = "exact",
                         want=("hit_id", "dist", "pos", "rgb"), out: dict | None = None) -> dict:
        """One whole frame: calculateScreen + shadeScreen (rt_render_frame).

        out: the dict a previous call returned, to write this frame into the
        same host arrays (runTest fills one global ray_hits vector frame after
        frame, src/main.cpp:39,322-349); `want` is then taken from it."""
        npx = int(W) * int(H)
        if out is not None:
            spec = {"hit_id": ((npx,), np.uint32), "dist": ((npx,), np.float64), "pos": ((npx, 3), np.float64),
                    "rgb": ((npx, 3), np.uint8)}
            for k, (shp, dt) in spec.items():
                a = out.get(k)
                if a is not None and (a.shape != shp or a.dtype != dt or not a.flags.c_contiguous):
                    raise ValueError(f"out[{k!r}] must be a C-contiguous {np.dtype(dt).name} array of shape {shp}")
        else:
            out = {"hit_id": np.empty(npx, np.uint32) if "hit_id" in want else None,
                   "dist": np.empty(npx) if "dist" in want else None,
                   "pos": np.empty((npx, 3)) if "pos" in want else None,
                   "rgb": np.empty((npx, 3), np.uint8) if "rgb" in want else None}
        fo = N.rt_frame_out()
        if out["hit_id"] is not None:
            fo.hit_id = out["hit_id"].ctypes.data_as(C.POINTER(C.c_uint32))
        if out["dist"] is not None:
            fo.dist = _dp(out["dist"])
        if out["pos"] is not None:
            fo.pos = _dp(out["pos"])
        if out["rgb"] is not None:
            fo.rgb = out["rgb"].ctypes.data_as(C.POINTER(C.c_uint8))
        cam = _camera(pos, d, W, H)
        m = N.RT_MODE_FP64 if mode in ("fp64", "literal") else N.RT_MODE_EXACT
        N.check(N.lib().rt_render_frame(self._h, C.byref(cam), m, C.byref(fo)))
        out["hits"] = int(fo.hit_count)
        out["seconds"] = float(fo.seconds)
        return out

    render = calculate_screen

    def render_rows_device(self, device: int, pos, d, W: int, H: int, row0: int, row_stride: int, nrows: int,
                           hit_id=0, dist=0, hit_pos=0, rgb=0, hit_count=0, stream=0, mode: str = "exact",
                           count: bool = False, timing: bool = False):
        """Asynchronous shard render into device pointers (ints) on `stream`.

        count: accumulate fetch counters; timing: time the pipeline kernels with
        HIP events on the library's launch stream (both read by frame_stats)."""
        o = N.rt_device_out(hit_id or None, dist or None, hit_pos or None, rgb or None, hit_count or None)
        cam = _camera(pos, d, W, H)
        m = N.RT_MODE_FP64 if mode in ("fp64", "literal") else N.RT_MODE_EXACT
        N.check(N.lib().rt_render_rows_device(self._h, int(device), C.byref(cam), m, int(row0), int(row_stride),
                                              int(nrows), C.byref(o), C.c_void_p(stream or None),
                                              (N.RT_FLAG_COUNT if count else 0) |
                                              (N.RT_FLAG_TIMING if timing else 0)))

    def render_batch_device(self, device: int, cams, W: int, H: int, row0: int, row_stride: int, nrows: int,
                            hit_id=0, dist=0, hit_pos=0, rgb=0, hit_count=0, stream=0, mode: str = "exact",
                            count: bool = False, timing: bool = False, spp: int = 1, counts_store: bool = False):
        """Asynchronous shard render of several poses ``cams`` = [(pos, dir), ...]
        (runTest's camera loop, src/main.cpp:234-281) into device pointers: pose
        f's outputs start f * W * nrows pixels in (per-sample outputs: times spp),
        its hit counter is hit_count[f] (added to; counts_store: set,
        RT_FLAG_COUNTS_STORE).  spp = n*n stratified samples per pixel
        (include/rt.h rt_render_batch_spp_device)."""
        n = len(cams)
        arr = (N.rt_camera * max(n, 1))(*[_camera(p, d, W, H) for p, d in cams])
        o = N.rt_device_out(hit_id or None, dist or None, hit_pos or None, rgb or None, hit_count or None)
        m = N.RT_MODE_FP64 if mode in ("fp64", "literal") else N.RT_MODE_EXACT
        N.check(N.lib().rt_render_batch_spp_device(self._h, int(device), arr, n, int(spp), m, int(row0),
                                                   int(row_stride), int(nrows), C.byref(o),
                                                   C.c_void_p(stream or None),
                                                   (N.RT_FLAG_COUNT if count else 0) |
                                                   (N.RT_FLAG_TIMING if timing else 0) |
                                                   (N.RT_FLAG_COUNTS_STORE if counts_store else 0)))

    def render_shard_device(self, device: int, cams, W: int, H: int, shard: int, nshards: int, hit_id=0, dist=0,
                            hit_pos=0, rgb=0, hit_count=0, stream=0, mode: str = "exact", count: bool = False,
                            timing: bool = False, spp: int = 1, job: dict | None = None, side_slot: bool = False,
                            counts_store: bool = False):
        """Shard `shard` of `nshards` of every pose (bands of 8 rows interleaved,
        include/rt.h rt_render_shard_device) into device pointers: pose f's
        outputs start f * W * shard_height(H, nshards, shard) pixels in.
        job: the fields of an rt_deinterleave_job (gathered, block_bytes,
        section_offset, shards, frames, height, width, elem_bytes, frame_rows,
        frames_out) carried out on the side by this render's kernel
        (rt_render_shard_device_job).  side_slot: RT_FLAG_SIDE_SLOT (one
        workgroup slot per CU left free for a collective on another stream);
        counts_store: RT_FLAG_COUNTS_STORE (hit_count[f] set, not added to)."""
        n = len(cams)
        arr = (N.rt_camera * max(n, 1))(*[_camera(p, d, W, H) for p, d in cams])
        o = N.rt_device_out(hit_id or None, dist or None, hit_pos or None, rgb or None, hit_count or None)
        m = N.RT_MODE_FP64 if mode in ("fp64", "literal") else N.RT_MODE_EXACT
        fl = ((N.RT_FLAG_COUNT if count else 0) | (N.RT_FLAG_TIMING if timing else 0) |
              (N.RT_FLAG_SIDE_SLOT if side_slot else 0) | (N.RT_FLAG_COUNTS_STORE if counts_store else 0))
        if job is None:
            N.check(N.lib().rt_render_shard_device(self._h, int(device), arr, n, int(spp), m, int(shard),
                                                   int(nshards), C.byref(o), C.c_void_p(stream or None), fl))
        else:
            j = N.rt_deinterleave_job(**job)
            N.check(N.lib().rt_render_shard_device_job(self._h, int(device), arr, n, int(spp), m, int(shard),
                                                       int(nshards), C.byref(o), C.byref(j),
                                                       C.c_void_p(stream or None), fl))

    def render_batch_multi(self, cams, W: int, H: int, hit_id=0, dist=0, hit_pos=0, rgb=0, hit_count=0, stream=0,
                           mode: str = "exact", count: bool = False, timing: bool = False, spp: int = 1,
                           counts_store: bool = False):
        """Full frames of every pose in ``cams`` over all uploaded devices (rows
        interleaved, RCCL gather to the first device, de-interleaved there) into
        device pointers on the first device (include/rt.h rt_render_batch_multi)."""
        n = len(cams)
        arr = (N.rt_camera * max(n, 1))(*[_camera(p, d, W, H) for p, d in cams])
        o = N.rt_device_out(hit_id or None, dist or None, hit_pos or None, rgb or None, hit_count or None)
        m = N.RT_MODE_FP64 if mode in ("fp64", "literal") else N.RT_MODE_EXACT
        N.check(N.lib().rt_render_batch_multi(self._h, arr, n, int(spp), m, C.byref(o), C.c_void_p(stream or None),
                                              (N.RT_FLAG_COUNT if count else 0) | (N.RT_FLAG_TIMING if timing else 0) |
                                              (N.RT_FLAG_COUNTS_STORE if counts_store else 0)))

    def render_paths_device(self, device: int, pos, d, W: int, H: int, row0: int, row_stride: int, nrows: int,
                            frame: int = 0, spp: int = 16, bounces: int = 4, hit_id=0, dist=0, hit_pos=0, rgb=0,
                            hit_count=0, stream=0, timing: bool = False, count: bool = False,
                            shadow: bool = False, counts_store: bool = False):
        """Diffuse path tracing of one pose into device pointers (include/rt.h
        rt_render_paths_device): rgb per pixel, primary-segment outputs per sample;
        count: add the ray segments traced to frame_stats()["rays"]; shadow: an
        occlusion ray toward the head-light from every bounce vertex
        (RT_FLAG_SHADOW); counts_store: hit_count set, not added to."""
        o = N.rt_device_out(hit_id or None, dist or None, hit_pos or None, rgb or None, hit_count or None)
        cam = _camera(pos, d, W, H)
        N.check(N.lib().rt_render_paths_device(self._h, int(device), C.byref(cam), int(frame), int(spp), int(bounces),
                                               int(row0), int(row_stride), int(nrows), C.byref(o),
                                               C.c_void_p(stream or None),
                                               (N.RT_FLAG_TIMING if timing else 0) | (N.RT_FLAG_COUNT if count else 0) |
                                               (N.RT_FLAG_SHADOW if shadow else 0) |
                                               (N.RT_FLAG_COUNTS_STORE if counts_store else 0)))

    def frame_stats(self, device: int = 0, reset: bool = True) -> dict:
        s = N.rt_frame_stats_t()
        N.check(N.lib().rt_frame_stats(self._h, int(device), int(reset), C.byref(s)))
        out = {}
        for f, _ in s._fields_:
            v = getattr(s, f)
            out[f] = list(v) if isinstance(v, C.Array) else v
        return out


def shard_height(H: int, nshards: int, shard: int) -> int:
    """Rows of one shard of the multi-GPU partition (include/rt.h rt_shard_height)."""
    return int(N.lib().rt_shard_height(int(H), int(nshards), int(shard)))


def deinterleave_rows(gathered: np.ndarray, shards: int, frames: int, H: int, W: int, elem_bytes: int,
                      block_bytes: int | None = None, section_offset: int = 0) -> np.ndarray:
    """Host de-interleave of gathered row shards (include/rt.h rt_deinterleave_rows):
    uint8 [frames, H, W * elem_bytes]."""
    g = np.ascontiguousarray(gathered, dtype=np.uint8).reshape(-1)
    block = len(g) // shards if block_bytes is None else int(block_bytes)
    out = np.empty((frames, H, W * elem_bytes), np.uint8)
    N.check(N.lib().rt_deinterleave_rows(g.ctypes.data, block, int(section_offset), int(shards), int(frames), int(H),
                                         int(W), int(elem_bytes), out.ctypes.data))
    return out


def ppm_bytes(rgb: np.ndarray, W: int, H: int) -> bytes:
    """PPM P6 bytes as Benchmark::saveScreen writes them (src/utils/benchmark.hpp:88-117)."""
    return f"P6\n{W} {H}\n255\n".encode() + np.ascontiguousarray(rgb, dtype=np.uint8).reshape(H, W, 3).tobytes()
