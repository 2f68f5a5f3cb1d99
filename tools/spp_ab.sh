set -u
cd "${GRAFT_REPO_ROOT:-.}"
for c in "RT_SPP_PACK=0" "RT_SPP_PACK=1" "RT_SPP_PACK=0" "RT_SPP_PACK=1"; do
  env $c timeout -k 10 300 python bench.py --no-cpu --steps 5 --spp 4 > gpurun_out/spp_$c.log 2>&1 || { echo "FAIL $c"; tail -5 gpurun_out/spp_$c.log; exit 1; }
  python -c "import json; l=[x for x in open('gpurun_out/spp_$c.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; q=r['per_ray']; print('RESULT', '$c', d['value'], r['kernel_ms_avg'], d['ms_per_step'], q['wave_nodes_per_tile'], q['wave_tris_per_tile'], q.get('redo_rays'))"
done
