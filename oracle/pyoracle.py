"""ctypes bindings for the TEST-ONLY checkers in oracle/.

    Oracle    -> oracle/build/librtoracle.so  (our CPU restatement, rt_oracle.cpp)
    Reference -> oracle/_ref/librtref.so      (reference headers compiled in place;
                                               present only where it was built)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The product package (raytracingdemo_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "librtoracle.so")
REF_SO = os.path.join(HERE, "_ref", "librtref.so")

ALGOS = {"median": 0, "sah": 1, "bsah": 2}

_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_longlong)


def build(quiet: bool = True) -> None:
    """Compile oracle/ (and oracle/_ref when /root/reference exists)."""
    out = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def _ptr(a, t):
    return None if a is None else a.ctypes.data_as(t)


def parse_algorithm(name: str):
    """'bsah' / 'bsah-c' / 'sah' / ... -> (algo id, collapse flag) (main.cpp:128-205)."""
    collapse = name.endswith("-c")
    base = name[:-2] if collapse else name
    if base not in ALGOS:
        raise ValueError(f"Unknown algorithm {name!r}")
    return ALGOS[base], collapse


class _Lib:
    def __init__(self, path: str, prefix: str):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (run oracle/Makefile)")
        self.lib = C.CDLL(path)
        self.p = prefix
        L, p = self.lib, prefix
        getattr(L, p + "last_error").restype = C.c_char_p
        f = getattr(L, p + "load_obj")
        f.argtypes = [C.c_char_p, C.c_double, C.POINTER(_dp)]
        f.restype = C.c_longlong
        getattr(L, p + "free").argtypes = [C.c_void_p]
        f = getattr(L, p + "scene_center")
        f.argtypes = [_dp, C.c_longlong, _dp]
        f = getattr(L, p + "camera_path")
        f.argtypes = [_dp, C.c_int, C.c_int, _dp, _dp]
        f = getattr(L, p + "bvh_create")
        f.argtypes = [_dp, C.c_longlong, C.c_int, C.c_int, C.c_int]
        f.restype = C.c_void_p
        getattr(L, p + "bvh_destroy").argtypes = [C.c_void_p]
        getattr(L, p + "bvh_dump").argtypes = [C.c_void_p, _dp, _i64p, _i64p]

    def err(self) -> str:
        return getattr(self.lib, self.p + "last_error")().decode()

    def load_obj(self, path: str, scale: float) -> np.ndarray:
        buf = _dp()
        n = getattr(self.lib, self.p + "load_obj")(path.encode(), float(scale), C.byref(buf))
        if n < 0:
            raise RuntimeError(self.err())
        arr = np.ctypeslib.as_array(buf, shape=(max(n, 1) * 9,))[: n * 9].copy().reshape(n, 9)
        getattr(self.lib, self.p + "free")(buf)
        return arr

    def scene_center(self, tris: np.ndarray) -> np.ndarray:
        t = np.ascontiguousarray(tris, dtype=np.float64)
        out = np.zeros(3)
        getattr(self.lib, self.p + "scene_center")(_ptr(t, _dp), len(t), _ptr(out, _dp))
        return out

    def camera_path(self, center, res: int, step: int):
        c = np.ascontiguousarray(center, dtype=np.float64)
        pos, d = np.zeros(3), np.zeros(3)
        getattr(self.lib, self.p + "camera_path")(_ptr(c, _dp), res, step, _ptr(pos, _dp), _ptr(d, _dp))
        return pos, d


@dataclass
class Tree:
    boxes: np.ndarray  # (nodes, 6) reference visit order
    meta: np.ndarray   # (nodes, 3) begin, end, nchildren
    order: np.ndarray  # owned primitive vector (loader indices)


class Oracle(_Lib):
    """Our CPU restatement of the reference path (rt_oracle.cpp)."""

    def __init__(self):
        super().__init__(ORACLE_SO, "orc_")
        L = self.lib
        L.orc_bvh_stats.argtypes = [C.c_void_p, _i64p]
        L.orc_render.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 _i32p, _dp, _dp, _dp, _u8p, C.POINTER(C.c_ulonglong)]
        L.orc_render.restype = C.c_longlong
        L.orc_render_spp.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     _i32p, _dp, _dp, _u8p]
        L.orc_render_spp.restype = C.c_longlong
        L.orc_render_paths.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_int, _i32p, _dp, _dp, _u8p, _i64p]
        L.orc_render_paths.restype = C.c_longlong
        L.orc_max_threads.restype = C.c_int

    def bvh(self, tris: np.ndarray, algorithm: str, k: int):
        return OracleBVH(self, tris, algorithm, k)

    def max_threads(self) -> int:
        return self.lib.orc_max_threads()


class OracleBVH:
    def __init__(self, lib: Oracle, tris: np.ndarray, algorithm: str, k: int):
        self.lib = lib
        self.tris = np.ascontiguousarray(tris, dtype=np.float64)
        algo, collapse = parse_algorithm(algorithm)
        self.h = lib.lib.orc_bvh_create(_ptr(self.tris, _dp), len(self.tris), algo, k, int(collapse))
        if not self.h:
            raise RuntimeError(lib.err())

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.lib.orc_bvh_destroy(self.h)
            self.h = None

    def stats(self) -> dict:
        out = np.zeros(5, dtype=np.int64)
        self.lib.lib.orc_bvh_stats(self.h, _ptr(out, _i64p))
        return dict(zip(["nodes", "inner", "leaves", "depth", "max_children"], out.tolist()))

    def dump(self) -> Tree:
        n = self.stats()["nodes"]
        boxes = np.zeros((n, 6))
        meta = np.zeros((n, 3), dtype=np.int64)
        order = np.zeros(len(self.tris), dtype=np.int64)
        self.lib.lib.orc_bvh_dump(self.h, _ptr(boxes, _dp), _ptr(meta, _i64p), _ptr(order, _i64p))
        return Tree(boxes, meta, order)

    def render(self, cam_pos, cam_dir, W: int, H: int, row0: int = 0, nrows: int | None = None,
               threads: int = 0, want=("id", "pos", "nrm", "dist", "rgb")):
        nrows = H - row0 if nrows is None else nrows
        n = W * nrows
        out = {}
        out["id"] = np.empty(n, np.int32) if "id" in want else None
        out["pos"] = np.empty((n, 3)) if "pos" in want else None
        out["nrm"] = np.empty((n, 3)) if "nrm" in want else None
        out["dist"] = np.empty(n) if "dist" in want else None
        out["rgb"] = np.empty((n, 3), np.uint8) if "rgb" in want else None
        cnt = (C.c_ulonglong * 3)()
        p = np.ascontiguousarray(cam_pos, dtype=np.float64)
        d = np.ascontiguousarray(cam_dir, dtype=np.float64)
        hits = self.lib.lib.orc_render(self.h, _ptr(p, _dp), _ptr(d, _dp), W, H, row0, nrows,
                                       threads or self.lib.max_threads(), _ptr(out["id"], _i32p),
                                       _ptr(out["pos"], _dp), _ptr(out["nrm"], _dp), _ptr(out["dist"], _dp),
                                       _ptr(out["rgb"], _u8p), cnt)
        if hits < 0:
            raise RuntimeError(self.lib.err())
        out["hits"] = int(hits)
        out["counters"] = tuple(int(c) for c in cnt)
        return out


    def render_spp(self, cam_pos, cam_dir, W: int, H: int, spp: int, row0: int = 0, nrows: int | None = None,
                   threads: int = 0):
        """Stratified spp = n*n samples per pixel (orc_render_spp): per-sample
        id / pos / dist ([pixels, spp]) and the averaged colour ([pixels, 3])."""
        nrows = H - row0 if nrows is None else nrows
        n = W * nrows
        out = {"id": np.empty((n, spp), np.int32), "pos": np.empty((n, spp, 3)), "dist": np.empty((n, spp)),
               "rgb": np.empty((n, 3), np.uint8)}
        p = np.ascontiguousarray(cam_pos, dtype=np.float64)
        d = np.ascontiguousarray(cam_dir, dtype=np.float64)
        hits = self.lib.lib.orc_render_spp(self.h, _ptr(p, _dp), _ptr(d, _dp), W, H, row0, nrows, int(spp),
                                           threads or self.lib.max_threads(), _ptr(out["id"], _i32p),
                                           _ptr(out["pos"], _dp), _ptr(out["dist"], _dp), _ptr(out["rgb"], _u8p))
        if hits < 0:
            raise RuntimeError(self.lib.err())
        out["hits"] = int(hits)
        return out


    def render_paths(self, cam_pos, cam_dir, W: int, H: int, frame: int, spp: int, bounces: int, row0: int = 0,
                     nrows: int | None = None, threads: int = 0, shadow: bool = False):
        """Diffuse paths (orc_render_paths): rgb per pixel, primary id / pos /
        dist per sample; shadow: head-light occlusion rays at the bounce
        vertices (shadow_cast / shadow_occluded counts)."""
        nrows = H - row0 if nrows is None else nrows
        n = W * nrows
        out = {"id": np.empty((n, spp), np.int32), "pos": np.empty((n, spp, 3)), "dist": np.empty((n, spp)),
               "rgb": np.empty((n, 3), np.uint8)}
        p = np.ascontiguousarray(cam_pos, dtype=np.float64)
        d = np.ascontiguousarray(cam_dir, dtype=np.float64)
        sc = np.zeros(2, dtype=np.int64)
        hits = self.lib.lib.orc_render_paths(self.h, _ptr(p, _dp), _ptr(d, _dp), W, H, row0, nrows, int(frame),
                                             int(spp), int(bounces), int(bool(shadow)),
                                             threads or self.lib.max_threads(),
                                             _ptr(out["id"], _i32p), _ptr(out["pos"], _dp), _ptr(out["dist"], _dp),
                                             _ptr(out["rgb"], _u8p), _ptr(sc, _i64p))
        if hits < 0:
            raise RuntimeError(self.lib.err())
        out["hits"] = int(hits)
        out["shadow_cast"], out["shadow_occluded"] = int(sc[0]), int(sc[1])
        return out


class Reference(_Lib):
    """The reference's own headers (oracle/_ref/librtref.so)."""

    def __init__(self):
        super().__init__(REF_SO, "ref_")
        L = self.lib
        L.ref_bvh_node_count.argtypes = [C.c_void_p]
        L.ref_bvh_node_count.restype = C.c_longlong
        L.ref_render.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 _u8p, _dp, _dp, _u8p]
        L.ref_render.restype = C.c_longlong

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def bvh(self, tris, algorithm: str, k: int):
        return RefBVH(self, tris, algorithm, k)


class RefBVH:
    def __init__(self, lib: Reference, tris, algorithm: str, k: int):
        self.lib = lib
        self.tris = np.ascontiguousarray(tris, dtype=np.float64)
        algo, collapse = parse_algorithm(algorithm)
        self.h = lib.lib.ref_bvh_create(_ptr(self.tris, _dp), len(self.tris), algo, k, int(collapse))
        if not self.h:
            raise RuntimeError(lib.err())

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.lib.ref_bvh_destroy(self.h)
            self.h = None

    def dump(self) -> Tree:
        n = self.lib.lib.ref_bvh_node_count(self.h)
        boxes = np.zeros((n, 6))
        meta = np.zeros((n, 3), dtype=np.int64)
        order = np.zeros(len(self.tris), dtype=np.int64)
        self.lib.lib.ref_bvh_dump(self.h, _ptr(boxes, _dp), _ptr(meta, _i64p), _ptr(order, _i64p))
        return Tree(boxes, meta, order)

    def render(self, cam_pos, cam_dir, W: int, H: int, row0: int = 0, nrows: int | None = None,
               threads: int = 8):
        nrows = H - row0 if nrows is None else nrows
        n = W * nrows
        hit = np.empty(n, np.uint8)
        pos = np.empty((n, 3))
        nrm = np.empty((n, 3))
        rgb = np.empty((n, 3), np.uint8)
        p = np.ascontiguousarray(cam_pos, dtype=np.float64)
        d = np.ascontiguousarray(cam_dir, dtype=np.float64)
        hits = self.lib.lib.ref_render(self.h, _ptr(p, _dp), _ptr(d, _dp), W, H, row0, nrows, threads,
                                       _ptr(hit, _u8p), _ptr(pos, _dp), _ptr(nrm, _dp), _ptr(rgb, _u8p))
        return {"hit": hit.astype(bool), "pos": pos, "nrm": nrm, "rgb": rgb, "hits": int(hits)}


def ppm_bytes(rgb: np.ndarray, W: int, H: int) -> bytes:
    """benchmark.hpp:88-117 byte layout: header then rows j, columns i."""
    return f"P6\n{W} {H}\n255\n".encode() + np.ascontiguousarray(rgb, dtype=np.uint8).reshape(H, W, 3).tobytes()
