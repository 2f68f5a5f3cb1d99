set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base w8k6; do
if [ $v = base ]; then L=""; else L=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so; fi
RT_LIB=$L timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/$v$rep.log 2>&1 || exit 1
done; done
grep -o '"value": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/base*.log gpurun_out/w8k6*.log
