set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --paths --no-cpu --steps 2 --warmup 1 > gpurun_out/p_base.log 2>&1 && tail -1 gpurun_out/p_base.log | cut -c1-160 || exit 1
for v in w4s8 w5s8 w6s8; do
RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so timeout -k 10 300 python bench.py --paths --no-cpu --steps 2 --warmup 1 > gpurun_out/p_$v.log 2>&1 && echo $v && tail -1 gpurun_out/p_$v.log | cut -c1-160 || exit 1
done
