"""rtdemo (the reference runner on the C ABI) against the reference's goldens.

rtdemo reproduces main.cpp's runTest output: testruns/testrun_<n>/ with
bvh_build_times.csv, render_times.csv, shading_times.csv and screen_<k>.ppm.
Its PPM bytes, hit counts and camera strings must equal the reference's
published testruns_final/ (tests/golden/reference_frames.json), and the CSV
layout must be the one scripts/validate_data.py reads.  The OBJ inputs are
written from the golden triangle soups (the reference's example/ is not on
the GPU box); objl reads them back to the same soup.
"""
from __future__ import annotations

import csv
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLD, ROOT

pytestmark = pytest.mark.gpu

DEMO = os.path.join(ROOT, "raytracingdemo_amd", "rtdemo")
HEADER = ["file_name", "model_name", "model_scale", "algorithm_name", "cam_pos_x", "cam_pos_y", "cam_pos_z",
          "cam_dir_x", "cam_dir_y", "cam_dir_z", "time_seconds"]


def _write_obj(model: str, path: str) -> None:
    z = np.load(os.path.join(GOLD, "scenes", model.replace(".obj", ".npz")))
    with open(path, "w") as f:
        f.write("".join(f"v {x:.9g} {y:.9g} {w:.9g}\n" for x, y, w in z["verts"].tolist()))
        f.write("".join(f"f {a + 1} {b + 1} {c + 1}\n" for a, b, c in z["idx"].reshape(-1, 3).tolist()))


def _rows(path):
    with open(path) as f:
        r = csv.reader(f)
        header = next(r)
        return header, list(r)


def test_rtdemo_reproduces_reference_testruns(tmp_path, frames_golden):
    if not os.path.exists(DEMO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracingdemo_amd", "csrc")], check=True)
    objects = tmp_path / "example"
    objects.mkdir()
    models = ["suzanne.obj", "teapot.obj"]
    for m in models:
        _write_obj(m, str(objects / m))
    out = tmp_path / "testruns"
    algos = ["bsah-2", "sah-c-8"]
    subprocess.run([DEMO, "--objects", str(objects), "--out", str(out), "--reps", "1", "--algos", ",".join(algos),
                    "--models", ",".join(models), "--frames", "36", "--size", "500"], check=True,
                   stdout=subprocess.DEVNULL, timeout=900)
    runs = sorted(out.iterdir(), key=lambda p: int(p.name.split("_")[1]))
    # sweep order: algorithms outer, models inner (std::map order), one run each
    assert [p.name for p in runs] == [f"testrun_{i}" for i in range(len(algos) * len(models))]
    first_ppm = {}
    for n, run in enumerate(runs):
        algo, model = algos[n // len(models)], models[n % len(models)]
        g = frames_golden[model]
        header, build = _rows(run / "bvh_build_times.csv")
        assert header == HEADER and len(build) == 10
        assert all(r[0] == "bvh_build_times.csv" and r[1] == model and r[3] == algo for r in build)
        header, shade = _rows(run / "shading_times.csv")
        assert header == HEADER and len(shade) == 36
        header, times = _rows(run / "render_times.csv")
        assert header == HEADER and len(times) == 36 and all(float(r[10]) > 0 for r in times)
        for k, (row, f) in enumerate(zip(shade, g["frames"])):
            assert row[4:7] == f["cam_pos"] and row[7:10] == f["cam_dir"], (model, k)
            assert row[10] == str(f["hits"]), (model, k)   # hit count printed as a double
            ppm = (run / f"screen_{k}.ppm").read_bytes()
            assert hashlib.sha256(ppm).hexdigest() == f["sha256"], (model, algo, k)
            # validate_data.py's invariant: every algorithm renders the same bytes
            first_ppm.setdefault((model, k), ppm)
            assert first_ppm[(model, k)] == ppm
        assert row[2] == ("3" if model == "suzanne.obj" else "1")  # model_scale, ostream default format
