set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_nohoist.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t2.log 2>&1; rc=$?; tail -2 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/r$rep.log 2>&1 && tail -1 gpurun_out/r$rep.log | cut -c1-140 || exit 1
done
grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/r*.log
