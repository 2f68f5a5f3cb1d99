set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --paths --steps 2 --warmup 1 > gpurun_out/paths_bench.log 2>&1 && tail -1 gpurun_out/paths_bench.log | cut -c1-200
