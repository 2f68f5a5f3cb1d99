#!/usr/bin/env bash
# Samples the GPU shader clock (rocm-smi) while a bench runs, plus the
# GRBM_GUI_ACTIVE-based effective clock of the traversal kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/clock_bench.log 2>&1 &
BP=$!
for k in $(seq 1 12); do
    sleep 2
    timeout 20 rocm-smi --showclocks --showpower --showtemp >> gpurun_out/clock_smi.log 2>&1 || true
done
wait $BP
echo "bench exit=$?"
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clk -o clk \
    -- python bench.py --steps 1 --warmup 0 --frames 4 --no-cpu > gpurun_out/clock_pmc.log 2>&1
echo "pmc exit=$?"
