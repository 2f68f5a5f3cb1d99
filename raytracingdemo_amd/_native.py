"""ctypes binding of librtmi355x.so (include/rt.h).

The shared library is built in-tree (raytracingdemo_amd/librtmi355x.so) by
``__graft_entry__.build()`` / ``make -C raytracingdemo_amd/csrc``.  There is no
fallback: if the library is missing or no gfx950 device is present, calls fail
loudly with :class:`RTError`.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RT_LIB selects an in-tree tuning build (raytracingdemo_amd/variants/) for A/B runs.
LIB_PATH = os.environ.get("RT_LIB") or os.path.join(HERE, "librtmi355x.so")

# include/rt.h status codes
RT_OK = 0
RT_ERR_INVALID_ARGUMENT = 1
RT_ERR_OUT_OF_RANGE = 2
RT_ERR_RUNTIME = 3
RT_ERR_HIP = 4
RT_ERR_NO_DEVICE = 5
STATUS_NAMES = {1: "invalid_argument", 2: "out_of_range", 3: "runtime_error", 4: "hip_error", 5: "no_device"}

RT_MODE_EXACT = 0
RT_MODE_FP64 = 1
RT_FLAG_COUNT = 1
RT_FLAG_TIMING = 2
RT_FLAG_SHADOW = 4
RT_FLAG_SIDE_SLOT = 8
RT_FLAG_COUNTS_STORE = 16
RT_MISS = 0xFFFFFFFF

# Every symbol include/rt.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "rt_load_obj", "rt_load_obj_cached", "rt_free", "rt_scene_center", "rt_camera_path", "rt_scene_create", "rt_scene_upload",
    "rt_render_frame", "rt_render_rows_device", "rt_render_batch_device", "rt_render_batch_spp_device", "rt_render_paths_device", "rt_frame_stats", "rt_scene_stats", "rt_scene_tree_dump",
    "rt_scene_destroy", "rt_last_error", "rt_abi_version", "rt_device_name", "rt_diag_raw",
    "rt_render_batch_multi", "rt_deinterleave_rows", "rt_scene_create_on_device", "rt_scene_build_times",
    "rt_render_shard_device", "rt_shard_height", "rt_render_shard_device_job", "rt_rccl_path",
]


class RTError(RuntimeError):
    """A non-OK status from the C ABI (the reference would have thrown)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"[{STATUS_NAMES.get(status, status)}] {msg}")
        self.status = status
        self.msg = msg


class rt_camera(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("dir", C.c_double * 3), ("width", C.c_int32), ("height", C.c_int32)]


class rt_frame_out(C.Structure):
    _fields_ = [("hit_id", C.POINTER(C.c_uint32)), ("dist", C.POINTER(C.c_double)), ("pos", C.POINTER(C.c_double)),
                ("rgb", C.POINTER(C.c_uint8)), ("hit_count", C.c_uint64), ("seconds", C.c_double)]


class rt_device_out(C.Structure):
    _fields_ = [("hit_id", C.c_void_p), ("dist", C.c_void_p), ("pos", C.c_void_p), ("rgb", C.c_void_p),
                ("hit_count", C.c_void_p)]


class rt_deinterleave_job(C.Structure):
    _fields_ = [("gathered", C.c_void_p), ("block_bytes", C.c_uint64), ("section_offset", C.c_uint64),
                ("shards", C.c_int), ("frames", C.c_int), ("height", C.c_int), ("width", C.c_int),
                ("elem_bytes", C.c_int), ("frame_rows", C.c_int), ("frames_out", C.c_void_p)]


class rt_scene_stats_t(C.Structure):
    _fields_ = [("triangles", C.c_uint64), ("real_nodes", C.c_uint64), ("real_inner", C.c_uint64),
                ("real_leaves", C.c_uint64), ("depth", C.c_uint32), ("max_children", C.c_uint32),
                ("max_leaf_size", C.c_uint32), ("wide_width", C.c_uint32), ("wide_nodes", C.c_uint64),
                ("device_bytes", C.c_uint64), ("stack_bound", C.c_uint32), ("node_bytes", C.c_double),
                ("walk_tree", C.c_uint32), ("layout_digest", C.c_uint64)]


class rt_frame_stats_t(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_fetches", C.c_uint64), ("tri_tests", C.c_uint64),
                ("chain_checks", C.c_uint64), ("hits", C.c_uint64), ("chain_nodes", C.c_uint64),
                ("tri_prefilter", C.c_uint64), ("wave_nodes", C.c_uint64), ("wave_leaves", C.c_uint64),
                ("wave_tiles", C.c_uint64), ("wave_tris", C.c_uint64), ("redo_rays", C.c_uint64), ("redo_chain", C.c_uint64),
                ("spilled_rays", C.c_uint64), ("dropped_rays", C.c_uint64), ("empty_node_steps", C.c_uint64),
                ("wave_tri_tests", C.c_uint64), ("wave_winners", C.c_uint64),
                ("shadow_rays", C.c_uint64), ("shadow_occluded", C.c_uint64),
                ("side_jobs_fused", C.c_uint64), ("side_jobs_kernel", C.c_uint64),
                ("shadow_wave_nodes", C.c_uint64), ("shadow_wave_tris", C.c_uint64),
                ("shadow_lane_nodes", C.c_uint64), ("shadow_lane_tris", C.c_uint64), ("timed_launches", C.c_uint64), ("trace_ms", C.c_double),
                ("lane_wave_nodes", C.c_uint64), ("lane_wave_tris", C.c_uint64)]


class rt_build_times_t(C.Structure):
    _fields_ = [("soup_ms", C.c_double), ("reference_tree_ms", C.c_double), ("walk_tree_ms", C.c_double),
                ("flatten_ms", C.c_double), ("walk_device", C.c_int32), ("reserved", C.c_int32),
                ("total_ms", C.c_double)]


_lib = None


def _share_hip_runtime_with_torch() -> None:
    """One HIP runtime per process.

    PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, loaded by
    torch as "libamdhip64.so" from torch/lib).  If librtmi355x.so were loaded
    first it would pull /opt/rocm's copy and torch would then map a second
    runtime that finds no GPU.  Pre-loading torch's file (RTLD_GLOBAL) makes
    our NEEDED libamdhip64.so.7 bind to it, and torch later reuses the same
    mapped file.  Without torch installed, /opt/rocm's runtime is used.
    """
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    # Only the HIP runtime: torch's librccl.so mapped RTLD_GLOBAL ahead of
    # `import torch` gets its static objects destroyed twice at exit ("double
    # free or corruption").  RCCL is dlopen'ed by soname (librccl.so.1) on the
    # first multi-device upload and so binds to torch's copy when torch is in.
    cand = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(cand):
        C.CDLL(cand, mode=C.RTLD_GLOBAL)


def lib() -> C.CDLL:
    """Load librtmi355x.so once (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RTError(RT_ERR_NO_DEVICE, f"{LIB_PATH} is not built (run __graft_entry__.build())")
    _share_hip_runtime_with_torch()
    L = C.CDLL(LIB_PATH)
    dp, u64p = C.POINTER(C.c_double), C.POINTER(C.c_uint64)
    L.rt_last_error.restype = C.c_char_p
    L.rt_device_name.restype = C.c_char_p
    L.rt_device_name.argtypes = [C.c_int]
    if hasattr(L, "rt_rccl_path"):
        L.rt_rccl_path.restype = C.c_char_p
    L.rt_abi_version.restype = C.c_int
    L.rt_load_obj.argtypes = [C.c_char_p, C.c_double, C.POINTER(dp), u64p]
    L.rt_free.argtypes = [C.c_void_p]
    L.rt_load_obj_cached.argtypes = [C.c_char_p, C.c_double, C.c_char_p, C.POINTER(dp), u64p, C.POINTER(C.c_int)]
    L.rt_scene_center.argtypes = [C.c_void_p, C.c_uint64, dp]
    L.rt_camera_path.argtypes = [dp, C.c_int, C.c_int, dp, dp]
    L.rt_scene_create.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.rt_scene_create_on_device.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.POINTER(C.c_void_p)]
    L.rt_scene_build_times.argtypes = [C.c_void_p, C.POINTER(rt_build_times_t)]
    L.rt_scene_upload.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    L.rt_render_frame.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.POINTER(rt_frame_out)]
    L.rt_render_rows_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.POINTER(rt_device_out), C.c_void_p, C.c_uint32]
    L.rt_render_batch_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.POINTER(rt_device_out), C.c_void_p, C.c_uint32]
    L.rt_render_batch_spp_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int, C.c_int, C.POINTER(rt_device_out), C.c_void_p,
                                             C.c_uint32]
    L.rt_render_paths_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_int, C.POINTER(rt_device_out), C.c_void_p, C.c_uint32]
    L.rt_render_shard_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.POINTER(rt_device_out), C.c_void_p, C.c_uint32]
    if hasattr(L, "rt_render_shard_device_job"):  # (RT_LIB tuning builds of earlier sources may lack it)
        L.rt_render_shard_device_job.argtypes = [C.c_void_p, C.c_int, C.POINTER(rt_camera), C.c_int, C.c_int,
                                                 C.c_int, C.c_int, C.c_int, C.POINTER(rt_device_out),
                                                 C.POINTER(rt_deinterleave_job), C.c_void_p, C.c_uint32]
    L.rt_shard_height.argtypes = [C.c_int, C.c_int, C.c_int]
    L.rt_render_batch_multi.argtypes = [C.c_void_p, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int,
                                        C.POINTER(rt_device_out), C.c_void_p, C.c_uint32]
    L.rt_deinterleave_rows.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_void_p]
    L.rt_frame_stats.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(rt_frame_stats_t)]
    L.rt_scene_stats.argtypes = [C.c_void_p, C.POINTER(rt_scene_stats_t)]
    L.rt_diag_raw.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
    L.rt_scene_tree_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.rt_scene_destroy.argtypes = [C.c_void_p]
    _lib = L
    return L


def prefer_torch_rccl() -> None:
    """Map PyTorch's RCCL before the library opens one (a multi-device
    upload), so the process holds one copy: the library reuses the mapped one
    (rt_api.cpp rccl())."""
    import importlib.util

    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401  (libtorch_hip maps torch/lib/librccl.so)


def check(status: int) -> None:
    if status != RT_OK:
        raise RTError(status, lib().rt_last_error().decode(errors="replace"))
