set -e
b() { timeout -k 10 300 python bench.py --no-cpu --steps 5 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r['per_ray']; print('$1', d['value'], r['trace_ms_per_frame'], r['frame_ms_avg'], p['wave_nodes_per_tile'])"; }
V=$PWD/raytracingdemo_amd/variants
RT_LIB=$V/librtmi355x_pc4.so timeout -k 10 300 python tools/node_fill.py
for rep in 1 2; do
b base
for v in k4 pc4 pc8; do RT_LIB=$V/librtmi355x_$v.so b $v; done
done
