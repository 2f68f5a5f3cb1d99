set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rtdemo.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/base$rep.log 2>&1 || exit 1
done
grep -o '"value": [0-9.]*' gpurun_out/base*.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp -o r -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/rp.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/rp/r_kernel_stats.csv')):
    if 'false>' in r['Name'] and ('resolve' in r['Name'] or 'packet' in r['Name']): print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3,'us')
"
