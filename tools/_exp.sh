set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/r2.log 2>&1 && tail -1 gpurun_out/r2.log | grep -o '"gather_verified": [a-z]*\|"n_gpus": [0-9]*' &&
RT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 7 --steps 3 --warmup 1 --frames 12 --no-cpu > gpurun_out/r7.log 2>&1 && tail -1 gpurun_out/r7.log | grep -o '"gather_verified": [a-z]*\|"n_gpus": [0-9]*'
