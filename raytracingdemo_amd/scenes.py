"""Synthetic workloads.

`sponza.obj` is stripped from the reference (/root/reference/.MISSING_LARGE_BLOBS:1),
so BASELINE.json's headline configuration runs on a deterministic procedural
**proxy**: a Crytek-Sponza-like atrium in centimetres with exactly 262,267
triangles (the count in example/object_meta.csv:6) — floor, two-storey
colonnades with arches, upper galleries, a third storey of slimmer columns,
curtains, spheres ("lion heads" / pots), outer walls with relief strips.  Its
triangle-centre mean sits in the open courtyard about 3.6 m up, like the real
scene's (testruns_2025_12_25/testrun_47/render_times.csv:2 camera
(-68.4, 364.9, -27.8)), so the reference's camera orbit (radius 5 around the
centre) looks across the courtyard into the colonnade.

Coordinates are rounded to float32 (what the OBJ loader would produce from a
file at scale 1).  If a real sponza.obj is supplied (env RT_SPONZA_OBJ), the
drivers use it instead and label it as such.
"""
from __future__ import annotations

import os

import numpy as np

SPONZA_TRIANGLES = 262267


def _grid(origin, u, v, nu, nv):
    o, u, v = (np.asarray(x, dtype=np.float64) for x in (origin, u, v))
    a = np.arange(nu + 1) / nu
    b = np.arange(nv + 1) / nv
    P = o + a[:, None, None] * u + b[None, :, None] * v  # (nu+1, nv+1, 3)
    p00, p10, p01, p11 = P[:-1, :-1], P[1:, :-1], P[:-1, 1:], P[1:, 1:]
    t1 = np.concatenate([p00, p10, p11], axis=-1).reshape(-1, 9)
    t2 = np.concatenate([p00, p11, p01], axis=-1).reshape(-1, 9)
    return np.concatenate([t1, t2])


def _surface(P):
    """Triangles of a parametric surface sampled as P[i, j, 3]."""
    p00, p10, p01, p11 = P[:-1, :-1], P[1:, :-1], P[:-1, 1:], P[1:, 1:]
    t1 = np.concatenate([p00, p10, p11], axis=-1).reshape(-1, 9)
    t2 = np.concatenate([p00, p11, p01], axis=-1).reshape(-1, 9)
    return np.concatenate([t1, t2])


def _cylinder(cx, y0, cz, r, h, nseg, nring, flute=0.0):
    th = np.linspace(0, 2 * np.pi, nseg + 1)
    y = np.linspace(y0, y0 + h, nring + 1)
    rr = r * (1 + flute * np.cos(12 * th))  # fluted column shaft
    X = cx + rr[:, None] * np.cos(th)[:, None] + 0 * y[None, :]
    Z = cz + rr[:, None] * np.sin(th)[:, None] + 0 * y[None, :]
    Y = np.broadcast_to(y[None, :], X.shape)
    return _surface(np.stack([X, Y, Z], axis=-1))


def _box(lo, hi, n=1):
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    faces = [_grid(lo, ex, ey, n, n), _grid(lo + ez, ey, ex, n, n), _grid(lo, ey, ez, n, n),
             _grid(lo + ex, ez, ey, n, n), _grid(lo, ez, ex, n, n), _grid(lo + ey, ex, ez, n, n)]
    return np.concatenate(faces)


def _sphere(c, r, nlat, nlon):
    th = np.linspace(0.05, np.pi - 0.05, nlat + 1)
    ph = np.linspace(0, 2 * np.pi, nlon + 1)
    X = c[0] + r * np.sin(th)[:, None] * np.cos(ph)[None, :]
    Y = c[1] + r * np.cos(th)[:, None] + 0 * ph[None, :]
    Z = c[2] + r * np.sin(th)[:, None] * np.sin(ph)[None, :]
    return _surface(np.stack([X, Y, Z], axis=-1))


def _arch(x0, x1, y_spring, z, depth, thick, nseg):
    """Semicircular arch band between two column axes at x0, x1 (plane z)."""
    cx, R = 0.5 * (x0 + x1), 0.5 * (x1 - x0)
    th = np.linspace(np.pi, 0, nseg + 1)
    out = []
    for rad in (R, R + thick):  # intrados and extrados
        X = cx + rad * np.cos(th)[:, None] + 0 * np.array([0, 1])[None, :]
        Y = y_spring + rad * np.sin(th)[:, None] + 0 * np.array([0, 1])[None, :]
        Z = z + np.array([-depth / 2, depth / 2])[None, :] + 0 * th[:, None]
        out.append(_surface(np.stack([X, Y, Z], axis=-1)))
    for zz in (z - depth / 2, z + depth / 2):  # the two faces
        rr = np.array([R, R + thick])
        X = cx + rr[None, :] * np.cos(th)[:, None]
        Y = y_spring + rr[None, :] * np.sin(th)[:, None]
        Z = np.full_like(X, zz)
        out.append(_surface(np.stack([X, Y, Z], axis=-1)))
    return np.concatenate(out)


def _curtain(x0, x1, y0, y1, z, amp, nu, nv, phase):
    u = np.linspace(0, 1, nu + 1)
    v = np.linspace(0, 1, nv + 1)
    X = x0 + (x1 - x0) * u[:, None] + 0 * v[None, :]
    Y = y1 - (y1 - y0) * v[None, :] + 0 * u[:, None]
    Z = z + amp * np.sin(2 * np.pi * 5 * u[:, None] + phase) * (0.3 + 0.7 * v[None, :])
    return _surface(np.stack([X, Y, Z], axis=-1))


def sponza_proxy_triangles(n_target: int = SPONZA_TRIANGLES) -> np.ndarray:
    """(n_target, 9) float64 triangle soup (float32-representable values).

    Deterministic; n_target < the full count scales the scene down for tests
    (fewer, coarser pieces) and still returns exactly n_target triangles.
    """
    s = min(1.0, n_target / SPONZA_TRIANGLES)
    q = lambda n: max(2, int(round(n * np.sqrt(s))))  # tessellation scale
    parts = []
    X0, X1, Z0, Z1 = -1900.0, 1800.0, -1100.0, 1150.0
    parts.append(_grid([X0, 0, Z0], [X1 - X0, 0, 0], [0, 0, Z1 - Z0], q(120), q(80)))       # floor
    for zs in (-1, 1):                                                                     # galleries
        zin, zout = (-460.0, Z0) if zs < 0 else (460.0, Z1)
        parts.append(_grid([X0, 600, zin], [X1 - X0, 0, 0], [0, 0, zout - zin], q(60), q(20)))
        parts.append(_grid([X0, 1100, zin], [X1 - X0, 0, 0], [0, 0, zout - zin], q(40), q(12)))
    parts.append(_grid([X0, 0, Z0], [X1 - X0, 0, 0], [0, 1500, 0], q(80), q(30)))            # outer walls
    parts.append(_grid([X0, 0, Z1], [0, 1500, 0], [X1 - X0, 0, 0], q(30), q(80)))
    parts.append(_grid([X0, 0, Z0], [0, 0, Z1 - Z0], [0, 1500, 0], q(50), q(30)))
    parts.append(_grid([X1, 0, Z0], [0, 1500, 0], [0, 0, Z1 - Z0], q(30), q(50)))
    xs = np.linspace(-1500, 1400, 9)
    for zc in (-460.0, 460.0):
        for lvl, (y0, h, r) in enumerate([(0, 520, 55), (600, 420, 45), (1100, 300, 30)]):
            for x in xs:
                parts.append(_cylinder(x, y0, zc, r, h, q(32), q(24), flute=0.04 if lvl < 2 else 0.0))
                parts.append(_box([x - r * 1.4, y0 + h - 30, zc - r * 1.4], [x + r * 1.4, y0 + h, zc + r * 1.4], q(3)))
                parts.append(_box([x - r * 1.3, y0, zc - r * 1.3], [x + r * 1.3, y0 + 25, zc + r * 1.3], q(2)))
            if lvl < 2:
                for a, b in zip(xs[:-1], xs[1:]):
                    parts.append(_arch(a, b, y0 + h, zc, 80.0, 40.0, q(40)))
        for k, (a, b) in enumerate(zip(xs[:-1], xs[1:])):                                 # curtains
            parts.append(_curtain(a + 50, b - 50, 640, 1000, zc + (25 if zc < 0 else -25), 18.0, q(40), q(30), 0.7 * k))
    for k, x in enumerate(np.linspace(-1400, 1300, 10)):                                   # lion heads / pots
        for zc in (-360.0, 360.0):
            parts.append(_sphere([x, 90 + 30 * (k % 3), zc], 70.0, q(24), q(32)))
    tris = np.concatenate(parts)
    n = len(tris)
    if n > n_target:
        tris = tris[:n_target]
    elif n < n_target:
        # relief strips on both long outer walls: small triangles 2 cm proud
        rest = n_target - n
        half = (rest + 1) // 2
        cols = max(1, int(np.ceil(np.sqrt(half / 2 * 8))))
        rows = int(np.ceil(half / 2 / cols))
        s0 = _grid([X0 + 100, 40, Z0 + 2.0], [X1 - X0 - 200, 0, 0], [0, 500, 0], cols, rows)[:half]
        s1 = _grid([X0 + 100, 40, Z1 - 2.0], [0, 500, 0], [X1 - X0 - 200, 0, 0], rows, cols)[: rest - half]
        tris = np.concatenate([tris, s0, s1])
    return _jitter(tris).astype(np.float32).astype(np.float64)


def _jitter(tris: np.ndarray, amp: float = 0.05) -> np.ndarray:
    """Deterministic per-vertex perturbation (shared vertices move together).

    The reference's binned SAH throws "invalid split position" when more than
    k primitives share one centre coordinate on a node's longest axis
    (stack_bvh.hpp:278-279 bins them all into bin 0, :542-543 throws); real
    scanned/modelled meshes never line up like the proxy's extruded bands do.
    """
    v = tris.reshape(-1, 3)
    key = np.round(v, 3)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    rng = np.random.Generator(np.random.PCG64(20260213))
    noise = rng.uniform(-amp, amp, size=(len(uniq), 3))
    return (v + noise[inv.reshape(-1)]).reshape(-1, 9)


def write_obj(tris: np.ndarray, path: str) -> None:
    """Write a triangle soup as OBJ (shared vertices, %.9g round-trips float32)."""
    f32 = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 3)
    verts, inv = np.unique(f32, axis=0, return_inverse=True)
    idx = inv.reshape(-1, 3) + 1
    with open(path, "w") as f:
        f.write(f"# sponza-proxy: {len(idx)} triangles (procedural stand-in, raytracingdemo_amd.scenes)\n")
        f.write("".join(f"v {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in verts.tolist()))
        f.write("".join(f"f {a} {b} {c}\n" for a, b, c in idx.tolist()))


def sponza_scene():
    """(triangles, label): the real sponza.obj if RT_SPONZA_OBJ names one, else the proxy."""
    path = os.environ.get("RT_SPONZA_OBJ")
    if path and os.path.exists(path):
        from . import load_obj
        return load_obj(path, 1.0), f"sponza.obj ({path})"
    return sponza_proxy_triangles(), "sponza-proxy (procedural, 262267 tris)"


ARMADILLO_SCALE = 0.035  # the reference runner's scale (testruns_2025_12_25/testrun_62/render_times.csv:2)


def armadillo_scene():
    """(triangles, label) of config c3 (armadillo.obj at the runner's scale
    0.035), or None: the geometry is stripped from the reference
    (.MISSING_LARGE_BLOBS), so it runs only where RT_ARMADILLO_OBJ names the
    file.  The reference's published frames of it (testruns_final/testrun_0)
    pin the result (tests/golden/reference_frames.json)."""
    path = os.environ.get("RT_ARMADILLO_OBJ")
    if not path or not os.path.exists(path):
        return None
    from . import load_obj
    return load_obj(path, ARMADILLO_SCALE), f"armadillo.obj ({path})"
