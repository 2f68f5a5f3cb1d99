set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/final_smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 &&
tail -2 gpurun_out/final_gpu_tests.log && tail -1 gpurun_out/final_smoke.log && tail -1 gpurun_out/final_bench.log | grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*'
