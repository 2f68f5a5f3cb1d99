set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for b in 12 18; do
RT_BATCH=$b timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/b$b_$rep.log 2>&1 || exit 1
cp gpurun_out/b$b_$rep.log gpurun_out/bt${b}_$rep.log
done; done
grep -o '"value": [0-9.]*' gpurun_out/bt*.log
