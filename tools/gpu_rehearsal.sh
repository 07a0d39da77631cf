# N>1 bench path rehearsed on the one GPU of a box: 2 and 4 processes, each a part of one sharded world
set -o pipefail
mkdir -p gpurun_out
RLO_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --ranks 64 --k 16384 > gpurun_out/bench2.log 2> gpurun_out/bench2.err && \
RLO_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --no-extras --ranks 64 --k 16384 > gpurun_out/bench4.log 2> gpurun_out/bench4.err
