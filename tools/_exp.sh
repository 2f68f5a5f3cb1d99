set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/h$rep.log 2>&1 && tail -1 gpurun_out/h$rep.log | cut -c1-140 &&
RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_nohoist.so timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/nh$rep.log 2>&1 && tail -1 gpurun_out/nh$rep.log | cut -c1-140 || exit 1
done
grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/h*.log gpurun_out/nh*.log
