set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base b36; do
if [ $v = base ]; then L=""; else L=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so; fi
RT_LIB=$L timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/$v$rep.log 2>&1 || exit 1
done; done
grep -o '"value": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/base*.log gpurun_out/b36*.log &&
RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_b36.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b36_gpu_tests.log 2>&1; tail -3 gpurun_out/b36_gpu_tests.log
