# A/B of the path kernel's packed samples (config c5): RT_PATHS_PACK=0 / 1, twice
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for c in "RT_PATHS_PACK=0" "RT_PATHS_PACK=1" "RT_PATHS_PACK=0" "RT_PATHS_PACK=1"; do
  env $c timeout -k 10 300 python bench.py --paths --no-cpu --steps 3 --warmup 1 > gpurun_out/paths_$c.log 2>&1 || { echo "FAIL $c"; tail -5 gpurun_out/paths_$c.log; exit 1; }
  python -c "import json; l=[x for x in open('gpurun_out/paths_$c.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('RESULT', '$c', d['value'], d['ms_per_step'], r['per_segment'])"
done
