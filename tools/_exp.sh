set -e
b() { timeout -k 10 300 python bench.py --no-cpu --paths --steps 2 --warmup 1 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['segments_traced_per_s_M'], d['kernel_ms_avg'])"; }
V=$PWD/raytracingdemo_amd/variants
b base
for v in p4 p5; do RT_LIB=$V/librtmi355x_$v.so b $v; done
