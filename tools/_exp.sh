set -e
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider 2>&1 | tail -4
b() { timeout -k 10 300 python bench.py --no-cpu --steps 5 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r['per_ray']; print('$1', d['value'], r['trace_ms_per_frame'], r['frame_ms_avg'], p['wave_nodes_per_tile'], p['wave_leaves_per_tile'], p['wave_tris_per_tile'], p['tri_tests_fp64'])"; }
b sah4
RT_WALK=ref b ref
RT_WALK_LEAF=2 b sah2
RT_WALK_LEAF=8 b sah8
