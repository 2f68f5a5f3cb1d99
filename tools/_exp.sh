set -e
b() { timeout -k 10 300 python bench.py --no-cpu --steps 5 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r['per_ray']; print('$1', d['value'], r['trace_ms_per_frame'], r['frame_ms_avg'])"; }
for rep in 1 2; do
b base
for v in c2 c3 w6; do RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so b $v; done
RT_WALK_LEAF=2 RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_c2.so b c2l2
done
