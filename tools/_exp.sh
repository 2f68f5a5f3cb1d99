set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --steps 5 > gpurun_out/b1.log 2>&1 && tail -1 gpurun_out/b1.log | cut -c1-400 &&
RT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/r2.log 2>&1 && tail -1 gpurun_out/r2.log | cut -c1-900 &&
RT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 3 --steps 3 --warmup 1 --no-cpu > gpurun_out/r3.log 2>&1 && tail -1 gpurun_out/r3.log | cut -c1-900
