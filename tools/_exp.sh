set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pwprof -o pw -- python bench.py --paths --no-cpu --steps 1 --warmup 0 > gpurun_out/pwprof.log 2>&1; echo rc=$?
cut -d, -f1-5 gpurun_out/pwprof/pw_kernel_stats.csv | head -12
