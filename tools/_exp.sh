set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paths" -p no:cacheprovider --timeout 300 > gpurun_out/tpaths.log 2>&1; rc=$?; tail -3 gpurun_out/tpaths.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --paths --no-cpu --steps 2 --warmup 1 > gpurun_out/pq.log 2>&1 && tail -1 gpurun_out/pq.log | cut -c1-200 &&
RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_noq.so timeout -k 10 300 python bench.py --paths --no-cpu --steps 2 --warmup 1 > gpurun_out/pn.log 2>&1 && tail -1 gpurun_out/pn.log | cut -c1-200
