#!/usr/bin/env python3
"""Regenerate tests/golden/ from the reference tree (run in the container that
has /root/reference; never at test time).

Writes
  golden/reference_frames.json  digests + hit counts of the reference's OWN
                                published frames (testruns_final/testrun_{0..3},
                                bsah-2; every algorithm yields the same bytes,
                                scripts/validate_data.py:21-72)
  golden/scenes/<model>.npz     the reference loader's triangle soup at scale 1
                                (ObjectLoader::loadFromFile, object_loader.hpp:14)
                                as float32 vertex table + int32 triangle indices
  golden/ref_trees.json         per (model, algorithm, k): tree statistics and a
                                sha256 of the reference's own tree dump
                                (StackBVH::build/collapse via oracle/_ref)
  golden/ref_pixels_<case>.npz  per-pixel outputs of the reference's
                                calculateScreen/shadeScreen (via oracle/_ref):
                                full rgb + hit mask, and hit position/normal
                                (fp64) on a strided pixel subset
"""
from __future__ import annotations

import csv
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

REF = os.environ.get("RT_REFERENCE", "/root/reference")
GOLD = os.path.join(ROOT, "tests", "golden")

# main.cpp:83-85 and the run index convention of testruns_final (model order
# is the std::map order: armadillo, bunny, suzanne, teapot).
MODELS = {"armadillo.obj": (0.035, 0), "stanford-bunny.obj": (30.0, 1), "suzanne.obj": (3.0, 2),
          "teapot.obj": (1.0, 3)}
# main.cpp:60-82 multimap order
ALGOS = [("bsah", 2), ("bsah", 4), ("bsah", 8), ("bsah", 16), ("bsah-c", 4), ("bsah-c", 8), ("bsah-c", 16),
         ("median", 2), ("median", 4), ("median", 8), ("median", 16), ("median-c", 4), ("median-c", 8),
         ("median-c", 16), ("sah", 2), ("sah", 4), ("sah", 8), ("sah", 16), ("sah-c", 4), ("sah-c", 8),
         ("sah-c", 16)]


def frames_json():
    out = {}
    for model, (scale, run) in MODELS.items():
        d = os.path.join(REF, "testruns_final", f"testrun_{run}")
        rows = list(csv.DictReader(open(os.path.join(d, "shading_times.csv"))))
        frames = []
        for step, r in enumerate(rows):
            ppm = open(os.path.join(d, f"screen_{step}.ppm"), "rb").read()
            frames.append({"step": step, "hits": int(float(r["time_seconds"])),
                           "cam_pos": [r["cam_pos_x"], r["cam_pos_y"], r["cam_pos_z"]],
                           "cam_dir": [r["cam_dir_x"], r["cam_dir_y"], r["cam_dir_z"]],
                           "md5": hashlib.md5(ppm).hexdigest(), "sha256": hashlib.sha256(ppm).hexdigest()})
        out[model] = {"scale": scale, "source": f"testruns_final/testrun_{run}", "algorithm": rows[0]["algorithm_name"],
                      "width": 500, "height": 500, "frames": frames}
    json.dump(out, open(os.path.join(GOLD, "reference_frames.json"), "w"), indent=1)


def tree_digest(t: pyoracle.Tree) -> str:
    h = hashlib.sha256()
    for a in (t.boxes, t.meta, t.order):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    os.makedirs(os.path.join(GOLD, "scenes"), exist_ok=True)
    frames_json()
    R = pyoracle.Reference()
    scenes = {}
    for model in ["teapot.obj", "suzanne.obj", "stanford-bunny.obj"]:
        tris = R.load_obj(os.path.join(REF, "example", model), 1.0)
        f32 = tris.astype(np.float32)
        assert np.array_equal(f32.astype(np.float64), tris)
        bits = np.ascontiguousarray(f32.reshape(-1, 3)).view(np.uint32)  # keep -0.0 distinct from 0.0
        ubits, inv = np.unique(bits, axis=0, return_inverse=True)
        verts = ubits.view(np.float32)
        idx = inv.reshape(-1, 3).astype(np.int32)
        assert verts[idx].reshape(-1, 9).tobytes() == f32.tobytes()
        np.savez_compressed(os.path.join(GOLD, "scenes", model.replace(".obj", ".npz")), verts=verts, idx=idx,
                            sha256=hashlib.sha256(tris.tobytes()).hexdigest())
        scenes[model] = tris
        print(model, tris.shape)

    trees = {}
    for model, tris1 in scenes.items():
        scale = MODELS[model][0]
        tris = tris1 * scale
        trees[model] = {"scale": scale, "tris_sha256": hashlib.sha256(tris.tobytes()).hexdigest(), "trees": {}}
        for algo, k in ALGOS:
            b = R.bvh(tris, algo, k)
            t = b.dump()
            nk = t.meta[:, 2]
            trees[model]["trees"][f"{algo}-{k}"] = {
                "nodes": int(len(t.meta)), "inner": int((nk > 0).sum()), "leaves": int((nk == 0).sum()),
                "max_children": int(nk.max()), "max_leaf": int((t.meta[nk == 0, 1] - t.meta[nk == 0, 0]).max()),
                "sha256": tree_digest(t)}
            print(model, algo, k, trees[model]["trees"][f"{algo}-{k}"]["nodes"])
    json.dump(trees, open(os.path.join(GOLD, "ref_trees.json"), "w"), indent=1)

    # per-pixel fixtures: (case, model, algo, k, W, H, step, stride)
    cases = [("c1_teapot_256_f0", "teapot.obj", "bsah", 2, 256, 256, 0, 7),
             ("suzanne_500_f5", "suzanne.obj", "bsah", 8, 500, 500, 5, 31),
             ("c2_bunny_1024_f0", "stanford-bunny.obj", "bsah", 4, 1024, 1024, 0, 97),
             ("bunny_640x360_f9", "stanford-bunny.obj", "sah-c", 8, 640, 360, 9, 53)]
    for name, model, algo, k, W, H, step, stride in cases:
        scale = MODELS[model][0]
        tris = scenes[model] * scale
        center = R.scene_center(tris)
        pos, d = R.camera_path(center, 36, step)
        b = R.bvh(tris, algo, k)
        r = b.render(pos, d, W, H)
        sel = np.arange(0, W * H, stride)
        np.savez_compressed(os.path.join(GOLD, f"ref_pixels_{name}.npz"), model=model, scale=scale, algo=algo, k=k,
                            W=W, H=H, step=step, cam_pos=pos, cam_dir=d, hits=r["hits"],
                            hit=np.packbits(r["hit"]), rgb=r["rgb"], sel=sel, pos=r["pos"][sel], nrm=r["nrm"][sel],
                            ppm_sha256=hashlib.sha256(pyoracle.ppm_bytes(r["rgb"], W, H)).hexdigest())
        print(name, r["hits"])


if __name__ == "__main__":
    main()
