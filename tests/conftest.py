"""Shared fixtures.  Markers: `gpu` = needs an MI355X (run with -m gpu)."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"  # only present in the build container, never on the GPU box
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

# scales of the reference runner (src/main.cpp:83-85)
SCALES = {"teapot.obj": 1.0, "suzanne.obj": 3.0, "stanford-bunny.obj": 30.0, "armadillo.obj": 0.035}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X (gfx950) device")


def golden_scene(model: str, scale: float | None = None) -> np.ndarray:
    """The reference loader's triangle soup for `model` (tests/golden/scenes), scaled
    exactly as ObjectLoader does (double(float) * scale)."""
    z = np.load(os.path.join(GOLD, "scenes", model.replace(".obj", ".npz")))
    tris = z["verts"][z["idx"]].reshape(-1, 9).astype(np.float64)
    s = SCALES[model] if scale is None else scale
    return tris * s


@pytest.fixture(scope="session")
def frames_golden():
    return json.load(open(os.path.join(GOLD, "reference_frames.json")))


@pytest.fixture(scope="session")
def trees_golden():
    return json.load(open(os.path.join(GOLD, "ref_trees.json")))


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    if not os.path.exists(pyoracle.ORACLE_SO):
        pyoracle.build()
    return pyoracle.Oracle()


def pixel_fixture(name: str):
    return np.load(os.path.join(GOLD, f"ref_pixels_{name}.npz"))


def pixel_fixture_names():
    return sorted(f[len("ref_pixels_"):-4] for f in os.listdir(GOLD) if f.startswith("ref_pixels_"))


def normals_of(tris: np.ndarray) -> np.ndarray:
    """Triangle normals with the reference's arithmetic (triangle.hpp:17)."""
    v0, v1, v2 = tris[:, 0:3], tris[:, 3:6], tris[:, 6:9]
    a, b = v1 - v0, v2 - v0
    n = np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                  a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], axis=1)
    ln = np.sqrt(n[:, 0] * n[:, 0] + n[:, 1] * n[:, 1] + n[:, 2] * n[:, 2])
    safe = np.where(ln == 0, 1.0, ln)
    return np.where(ln[:, None] == 0, 0.0, n / safe[:, None])
