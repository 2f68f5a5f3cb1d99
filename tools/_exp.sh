set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --paths --steps 2 --warmup 1 > gpurun_out/paths_bench.log 2>&1 && tail -1 gpurun_out/paths_bench.log | cut -c1-150 &&
timeout -k 10 300 python bench.py --spp 4 --no-cpu > gpurun_out/spp4_bench.log 2>&1 && tail -1 gpurun_out/spp4_bench.log | cut -c1-150
