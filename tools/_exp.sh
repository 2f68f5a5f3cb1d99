set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 -k "sponza or overflow or batch or reference" > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for v in base nopf; do
if [ $v = base ]; then L=""; else L=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so; fi
RT_LIB=$L timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/$v$rep.log 2>&1 || exit 1
done; done
grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/base*.log gpurun_out/nopf*.log
