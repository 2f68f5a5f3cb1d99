set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/demo_obj
python - <<'PY'
import numpy as np
z = np.load("tests/golden/scenes/teapot.npz")
with open("gpurun_out/demo_obj/teapot.obj", "w") as f:
    f.write("".join(f"v {x:.9g} {y:.9g} {w:.9g}\n" for x, y, w in z["verts"].tolist()))
    f.write("".join(f"f {a+1} {b+1} {c+1}\n" for a, b, c in z["idx"].reshape(-1, 3).tolist()))
PY
rm -rf gpurun_out/demo_testruns
timeout -k 10 300 ./raytracingdemo_amd/rtdemo --objects gpurun_out/demo_obj --out gpurun_out/demo_testruns --reps 1 --algos bsah-8,median-c-16 --models teapot.obj > gpurun_out/demo.log 2>&1
rm -rf gpurun_out/demo_obj
du -sh gpurun_out/demo_testruns
